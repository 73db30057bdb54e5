"""GPU: damc.optim (clip_grad_norm_ + Adam / AdamW on csrc/optim.hip) against torch.optim on the same tensors.

The reference's optimisers (workspace/train_gen_recon.py:155-157: Adam betas (0.5, 0.999) for G and E,
AdamW weight_decay=1e-4 for Q; clip_grad_norm_ before each step, :219/:230/:240) are the oracle here: the
same parameters, gradients and hyper-parameters go through torch's foreach implementation and through
the HIP kernels.  The HIP step follows torch's per-element op order and roundings; the tolerance below
(4 ulp-scale relative) covers the FMA contractions of torch's own ROCm kernels, which are not visible
from Python.  The clip norm is a different (fixed-order) summation: rel 1e-6.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(1024, 512, 4, 4), (512,), (3,), (5, 7), (8193,), (256, 3, 3, 3)]
STEP_TOL = 5e-7


def _params(device, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter((torch.randn(s, generator=g) * 0.05).to(device)) for s in SHAPES]


def _set_grads(params, step, scale=1.0):
    g = torch.Generator().manual_seed(100 + step)
    for p in params:
        p.grad = (torch.randn(p.shape, generator=g) * scale).to(p.device)


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("kind,kw", [
    ("adam", dict(lr=2e-4, betas=(0.5, 0.999))),                       # G / E optimiser
    ("adamw", dict(lr=3e-4, betas=(0.5, 0.999), weight_decay=1e-4)),   # Q optimiser
    ("adam", dict(lr=1e-3, weight_decay=1e-2)),                         # L2 form, default betas (lerp w < 0.5)
])
def test_adam_step_matches_torch(gpu_device, kind, kw):
    from damc import optim as dopt

    ref = _params(gpu_device)
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    tcls = torch.optim.Adam if kind == "adam" else torch.optim.AdamW
    dcls = dopt.Adam if kind == "adam" else dopt.AdamW
    to, do = tcls(ref, **kw), dcls(mine, **kw)
    for step in range(6):
        _set_grads(ref, step)
        _set_grads(mine, step)
        to.step()
        do.step()
    torch.cuda.synchronize()
    for a, b in zip(mine, ref):
        assert _rel(a.detach(), b.detach()) < STEP_TOL
        sa, sb = do.state[a], to.state[b]
        assert float(sa["step"]) == float(sb["step"]) == 6.0
        assert _rel(sa["exp_avg"], sb["exp_avg"]) < STEP_TOL
        assert _rel(sa["exp_avg_sq"], sb["exp_avg_sq"]) < STEP_TOL


@pytest.mark.parametrize("scale,max_norm", [(1.0, 1.0), (1e-3, 100.0)])  # clipping active / inactive
def test_clip_grad_norm_matches_torch(gpu_device, scale, max_norm):
    from damc import optim as dopt

    ref = _params(gpu_device)
    _set_grads(ref, 0, scale)
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    for a, b in zip(mine, ref):
        a.grad = b.grad.clone()
    tn = torch.nn.utils.clip_grad_norm_(ref, max_norm)
    dn = dopt.clip_grad_norm_(mine, max_norm)
    torch.cuda.synchronize()
    assert abs(float(dn) - float(tn)) / float(tn) < 1e-6
    for a, b in zip(mine, ref):
        assert _rel(a.grad, b.grad) < 1e-6


def test_clip_and_step_matches_torch_sequence(gpu_device):
    """The reference's `clip_grad_norm_(G.parameters(), g_max_norm); G_optimizer.step()` as one fused call."""
    from damc import optim as dopt

    ref = _params(gpu_device, seed=3)
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    to = torch.optim.Adam(ref, lr=2e-4, betas=(0.5, 0.999))
    do = dopt.Adam(mine, lr=2e-4, betas=(0.5, 0.999))
    for step in range(5):
        _set_grads(ref, step, scale=0.5)
        _set_grads(mine, step, scale=0.5)
        tn = torch.nn.utils.clip_grad_norm_(ref, 10.0)
        to.step()
        dn = do.clip_and_step(10.0)
        torch.cuda.synchronize()
        assert abs(float(dn) - float(tn)) / float(tn) < 1e-6
        for a, b in zip(mine, ref):
            assert _rel(a.grad, b.grad) < 1e-6  # gradients left scaled, as clip_grad_norm_ leaves them
    for a, b in zip(mine, ref):
        assert _rel(a.detach(), b.detach()) < 2e-6


def test_state_dict_interchanges_with_torch(gpu_device):
    """A torch Adam state (what the reference checkpoints) loads into damc.optim.Adam and continues identically."""
    from damc import optim as dopt

    ref = _params(gpu_device, seed=5)
    to = torch.optim.Adam(ref, lr=2e-4, betas=(0.5, 0.999))
    for step in range(3):
        _set_grads(ref, step)
        to.step()
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    do = dopt.Adam(mine, lr=2e-4, betas=(0.5, 0.999))
    do.load_state_dict(copy.deepcopy(to.state_dict()))
    for step in range(3, 5):
        _set_grads(ref, step)
        _set_grads(mine, step)
        to.step()
        do.step()
    torch.cuda.synchronize()
    for a, b in zip(mine, ref):
        assert _rel(a.detach(), b.detach()) < STEP_TOL
    back = torch.optim.Adam([torch.nn.Parameter(p.detach().clone()) for p in ref], lr=2e-4, betas=(0.5, 0.999))
    back.load_state_dict(do.state_dict())  # and back again
    assert float(back.state_dict()["state"][0]["step"]) == 5.0


def test_step_is_deterministic(gpu_device):
    from damc import optim as dopt

    outs = []
    for _ in range(2):
        ps = _params(gpu_device, seed=9)
        o = dopt.AdamW(ps, lr=1e-3, weight_decay=1e-4)
        for step in range(3):
            _set_grads(ps, step)
            o.clip_and_step(1.0)
        torch.cuda.synchronize()
        outs.append([p.detach().clone() for p in ps])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_more_tensors_than_one_launch(gpu_device):
    """130 parameters (> 96 per launch: two slices for the norm and the step) against torch."""
    from damc import optim as dopt

    g = torch.Generator().manual_seed(11)
    ref = [torch.nn.Parameter(torch.randn(int(n), generator=g).to(gpu_device))
           for n in torch.randint(1, 3000, (130,), generator=g)]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    to = torch.optim.AdamW(ref, lr=1e-3, betas=(0.5, 0.999), weight_decay=1e-4)
    do = dopt.AdamW(mine, lr=1e-3, betas=(0.5, 0.999), weight_decay=1e-4)
    for step in range(3):
        _set_grads(ref, step)
        _set_grads(mine, step)
        tn = torch.nn.utils.clip_grad_norm_(ref, 5.0)
        to.step()
        dn = do.clip_and_step(5.0)
        torch.cuda.synchronize()
        assert abs(float(dn) - float(tn)) / float(tn) < 1e-6
    for a, b in zip(mine, ref):
        assert _rel(a.detach(), b.detach()) < 2e-6


def test_adam_step_counters_with_partial_gradients(gpu_device):
    """damc.optim shares one step counter per group while every parameter is updated together (one CPU add per
    step instead of a foreach over ~100 scalars); a step in which only some parameters carry a gradient gives those
    their own counters first, so every parameter's count, its bias correction and the torch state_dict round trip
    still match torch's AdamW."""
    from damc import optim as dopt

    ref = _params(gpu_device)
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    kw = dict(lr=3e-4, betas=(0.5, 0.999), weight_decay=1e-4)
    to, do = torch.optim.AdamW(ref, **kw), dopt.AdamW(mine, **kw)
    for step in range(6):
        _set_grads(ref, step)
        _set_grads(mine, step)
        if step == 3:  # every other parameter without a gradient this step
            for i in range(0, len(ref), 2):
                ref[i].grad = None
                mine[i].grad = None
        to.step()
        do.step()
    torch.cuda.synchronize()
    for a, b in zip(mine, ref):
        assert float(do.state[a]["step"]) == float(to.state[b]["step"])
        assert _rel(a.detach(), b.detach()) < STEP_TOL
    # the state_dict carries the per-parameter counts into torch's optimiser and back
    to2 = torch.optim.AdamW(mine, **kw)
    to2.load_state_dict(do.state_dict())
    assert [float(to2.state[p]["step"]) for p in mine] == [float(to.state[p]["step"]) for p in ref]
    # ... and the stock optimiser keeps stepping from there exactly as torch's own (a shared counter in
    # the state_dict was advanced once per parameter by torch's step)
    _set_grads(ref, 6)
    _set_grads(mine, 6)
    to.step()
    to2.step()
    torch.cuda.synchronize()
    assert [float(to2.state[p]["step"]) for p in mine] == [float(to.state[p]["step"]) for p in ref]
    for a, b in zip(mine, ref):
        assert _rel(a.detach(), b.detach()) < STEP_TOL
