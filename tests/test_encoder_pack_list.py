"""CPU: the encoder's one-launch weight packing list (gemm.h PackConvList, gemm.hip pack_conv_x3_many_prep, the
device-side pack_conv_x3_block) restated on the host for every encoder the drivers build (diffusion_net.py:227-413 at
nif=64, nemb=1024): the prepared grid is exactly the work list -- every (layer, output channel, channel chunk) is
packed by exactly one workgroup, no workgroup falls outside the list, and a list prepared twice is refused (the
round-4 fault: a second preparation turned the running offsets into a grid larger than the list)."""
import pytest

ENC = {  # (hidden channel multipliers of nif, last kernel): src/diffusion_net.py _ENC_TOPOLOGY
    "cifar10": ((1, 2, 4, 8), 4),
    "celeba64": ((1, 2, 4, 8, 8), 4),
    "celebaHQ": ((1, 2, 4, 4, 8, 8, 8), 4),
}


def limb_layers(name, nif=64, nemb=1024, nc=3):
    """(cout, cin, taps) of the layers whose weights the library packs (Conv2d with cin % 64 == 0 or % 128 == 0)."""
    mults, kl = ENC[name]
    out, cin = [], nc
    for i, m in enumerate(mults):
        k = 3 if i == 0 else 4
        out.append((nif * m, cin, k * k))
        cin = nif * m
    out.append((nemb, cin, kl * kl))
    return [(co, ci, t) for co, ci, t in out if (ci % 128 == 0 or ci == 64) and t <= 32]


def prep(lst):
    """pack_conv_x3_many_prep: cc per layer, blk0 running workgroup offsets; refuses a prepared list."""
    if lst.get("ready"):
        raise ValueError("already prepared")
    cc = [128 if ci % 128 == 0 else 64 for _, ci, _ in lst["layers"]]
    blk0 = [0]
    for (co, ci, _), c in zip(lst["layers"], cc):
        blk0.append(blk0[-1] + co * (ci // c))
    total = sum(co * (ci // c) for (co, ci, _), c in zip(lst["layers"], cc))
    assert total == blk0[-1]
    lst.update(ready=True, cc=cc, blk0=blk0)
    return lst


def block(lst, blk):
    """pack_conv_x3_block's index math with its bound: (layer, co, cc0) or None (outside the list)."""
    layers, cc, blk0 = lst["layers"], lst["cc"], lst["blk0"]
    n = len(layers)
    if not lst.get("ready") or not (0 <= blk < blk0[n]):
        return None
    li = 0
    while li + 1 < n and blk >= blk0[li + 1]:
        li += 1
    b = blk - blk0[li]
    co_n, cin, _ = layers[li]
    nch = cin // cc[li]
    co, cc0 = b // nch, (b % nch) * cc[li]
    if co >= co_n or cc0 + cc[li] > cin:
        return None
    return li, co, cc0


@pytest.mark.parametrize("name", sorted(ENC))
def test_pack_grid_is_exactly_the_work_list(name):
    lst = prep({"layers": limb_layers(name)})
    seen = set()
    for blk in range(lst["blk0"][-1]):
        t = block(lst, blk)
        assert t is not None, blk
        assert t not in seen
        seen.add(t)
    want = {(li, co, c0) for li, (co_n, ci, _) in enumerate(lst["layers"]) for co in range(co_n)
            for c0 in range(0, ci, lst["cc"][li])}
    assert seen == want
    # a grid one workgroup larger than the list: the extra workgroup is outside it (the device bound returns early)
    assert block(lst, lst["blk0"][-1]) is None
    with pytest.raises(ValueError):
        prep(lst)
