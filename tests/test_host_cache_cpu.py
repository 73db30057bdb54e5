"""CPU: host-side plan caches and shape gates of damc.training (no kernel calls)."""
import torch

import conftest  # noqa: F401  (puts the package on sys.path)


def test_denoiser_param_cache_sees_a_replaced_submodule():
    """the per-denoiser parameter cache must notice ``blk._skip = nn.Linear(...)`` (the old module's
    parameter dict still holds the old tensors, so a check of those dicts alone hits the stale entry)."""
    from damc import training as T
    from src.diffusion_net import _netQ_U

    p = _netQ_U(nz=16, nxemb=32, ntemb=16, nif=8).p
    a = T._denoiser_params(p)
    assert T._denoiser_params(p) is a  # cached
    blk = T._blocks_of(p)[2]
    blk._skip = torch.nn.Linear(blk._skip.in_features, blk._skip.out_features)
    b = T._denoiser_params(p)
    assert b is not a
    assert any(t is blk._skip.weight for _, _, t in b) and any(t is blk._skip.bias for _, _, t in b)
    # a replaced Sequential member and a replaced block are seen too
    blk._layer_ctx[1] = torch.nn.Linear(blk._layer_ctx[1].in_features, blk._layer_ctx[1].out_features)
    c = T._denoiser_params(p)
    assert any(t is blk._layer_ctx[1].weight for _, _, t in c)


def test_ebm_layers_refuse_a_negative_slope():
    """the HIP E-update backward takes LReLU' from the post-activation's sign, valid for slopes >= 0 only;
    a negative slope keeps the stock modules."""
    from damc import training as T
    from src.diffusion_net import _netE

    E = _netE(nz=16, ndf=8)
    assert T._ebm_layers(E) is not None
    for m in E.ebm:
        if isinstance(m, torch.nn.LeakyReLU):
            m.negative_slope = -0.2
    assert T._ebm_layers(E) is None


def test_spectral_norm_step_is_one_reference_forward():
    """Train-mode spectral norm on the HIP chains (damc.plans.spectral_norm_step, diffusion_net.py:8-16): one step
    advances every layer's u and v exactly as one forward of the stock module does, sets the same normalised weight,
    and the plans read that weight only inside the step (outside it a train-mode layer is refused, so no chain can pack
    a weight whose power iteration did not run)."""
    import copy

    import pytest

    from damc import plans
    from src import diffusion_net as dn

    E = dn._netE(nz=16, ndf=24, e_sn=True).train()
    E2 = copy.deepcopy(E)
    ep = plans.ebm_plan(E)
    layers = ep.sn_train()
    assert len(layers) == 3
    z = torch.randn(4, 16)
    for _ in range(3):
        with plans.spectral_norm_step(layers):
            ws = [plans._live_weight(m).clone() for m in ep.lin]
        with torch.no_grad():
            E2.ebm(z)  # the stock forward: each SpectralNorm pre-hook runs one power iteration
        for m, m2, w in zip(ep.lin, [E2.ebm[0], E2.ebm[2], E2.ebm[4]], ws):
            assert torch.equal(m.weight_u, m2.weight_u) and torch.equal(m.weight_v, m2.weight_v)
            assert torch.equal(w, m2.weight)
    with pytest.raises(NotImplementedError):
        plans._live_weight(ep.lin[0])
    E.eval()
    assert ep.sn_train() == []
    w_eval = plans._live_weight(ep.lin[0])  # eval: no power iteration, the hook's weight
    with torch.no_grad():
        E2.eval().ebm(z)
    assert torch.equal(w_eval, E2.ebm[0].weight)
