"""CPU: host-side behaviour of damc.optim that needs no kernel (the state_dict a stock torch optimiser resumes from)."""
import io

import torch

import conftest  # noqa: F401  (puts the package on sys.path)


def test_state_dict_unshares_the_group_step_counter():
    """damc.optim keeps one ``step`` tensor per group (_advance_steps).  Its state_dict must give every
    parameter a private counter, or a stock AdamW that loads it (after torch.save / torch.load, which keep storage
    sharing) adds 1 to the shared tensor once per parameter and every bias correction after a resume is wrong."""
    from damc import optim as dopt

    torch.manual_seed(0)
    ref = [torch.nn.Parameter(torch.randn(5, 3)) for _ in range(4)]
    kw = dict(lr=1e-2, betas=(0.5, 0.999), weight_decay=1e-4)
    to = torch.optim.AdamW(ref, **kw)
    for _ in range(2):
        for p in ref:
            p.grad = torch.ones_like(p)
        to.step()
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    # the same two steps as damc.optim would leave them: the state of torch's run, with ONE shared step tensor
    do = dopt.AdamW(mine, **kw)
    shared = torch.tensor(2.0)
    for a, b in zip(mine, ref):
        st = to.state[b]
        do.state[a] = {"step": shared, "exp_avg": st["exp_avg"].clone(), "exp_avg_sq": st["exp_avg_sq"].clone()}
    sd = do.state_dict()
    steps = [v["step"] for v in sd["state"].values()]
    assert len({id(t) for t in steps}) == len(steps) and all(float(t) == 2.0 for t in steps)
    assert do.state[mine[0]]["step"] is shared  # the optimiser's own fast-path sharing is untouched
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    to2 = torch.optim.AdamW(mine, **kw)
    to2.load_state_dict(torch.load(buf, weights_only=True))
    for p in ref:
        p.grad = torch.ones_like(p)
    for p in mine:
        p.grad = torch.ones_like(p)
    to.step()
    to2.step()
    assert [float(to2.state[p]["step"]) for p in mine] == [3.0] * len(mine)
    for a, b in zip(mine, ref):
        assert torch.equal(a.detach(), b.detach())
