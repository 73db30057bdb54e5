"""GPU parity: the amortizer Q on the HIP path (encoder + prior embedding + reverse sweep) vs the
reference's golden vectors (workspace/src/diffusion_net.py:227-622).

Tolerances: encoder xemb rel-L2 <= 1e-5; eps of the first reverse step <= 1e-5, of steps 2-3 <= 1e-4
(inherited rounding, amplified by sqrt(1+e^-l) per step); end-point of the sweep <= conftest.Q_END_TOL
(2x the reference's own fp32-vs-fp64 spread on that case).
"""
import pytest
import torch

from conftest import Q_END_TOL, Q_NAMES, build_q_case, rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def am(gpu_device):
    from damc import amortizer

    return amortizer


@pytest.mark.parametrize("name", Q_NAMES)
def test_encoder_matches_reference(am, gpu_device, name):
    c = build_q_case(name, gpu_device)
    xemb = am.encoder_forward(c["Q"].encoder, c["x"])
    assert rel_l2(xemb.cpu().numpy(), c["rec"]["xemb"]) < 1e-5


@pytest.mark.parametrize("name", Q_NAMES)
def test_posterior_sweep_matches_reference(am, gpu_device, name):
    c = build_q_case(name, gpu_device)
    Q, rec = c["Q"], c["rec"]
    xemb = am.encoder_forward(Q.encoder, c["x"])
    zt = c["zt0"].clone()
    eps = am.reverse_sweep(Q, xemb, zt, noise=c["eps"], eps_log_steps=3).cpu().numpy()
    for k in range(3):
        assert rel_l2(eps[k], rec["q_post_eps3"][k]) < (1e-5 if k == 0 else 1e-4), k
    assert rel_l2(zt.cpu().numpy(), rec["q_post"]) < Q_END_TOL[name]


@pytest.mark.parametrize("name", Q_NAMES)
def test_prior_sweep_matches_reference(am, gpu_device, name):
    c = build_q_case(name, gpu_device)
    Q, rec = c["Q"], c["rec"]
    xemb = am.prior_embedding(Q, c["pe_noise"])
    zt = c["zt0"].clone()
    eps = am.reverse_sweep(Q, xemb, zt, noise=c["eps"], eps_log_steps=1).cpu().numpy()
    assert rel_l2(eps[0], rec["q_prior_eps3"][0]) < 1e-5
    assert rel_l2(zt.cpu().numpy(), rec["q_prior"]) < Q_END_TOL[name]


def test_denoise_step_vs_oracle_at_baseline_width(am, gpu_device):
    """Full-width CIFAR Q (nxemb=1024, ntemb=128) at B=128: first reverse step eps vs the fp32 oracle."""
    from damc import synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
    synth.load_into(Q, 20)
    Q.to(gpu_device).eval()
    B = 128
    x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, 32, 32))).to(gpu_device)
    zt0 = torch.from_numpy(synth.normal_f32(6, 0, (B, 128))).to(gpu_device)
    xemb = am.encoder_forward(Q.encoder, x)
    with torch.no_grad():
        xref = orc.encoder_forward(Q.encoder.cpu(), x.cpu())
        Q.to(gpu_device)
    assert rel_l2(xemb.cpu().numpy(), xref.numpy()) < 1e-5
    zt = zt0.clone()
    noise = torch.zeros(99, B, 128, device=gpu_device)
    eps = am.reverse_sweep(Q, xemb, zt, noise=noise, eps_log_steps=1)
    Qc = Q.cpu()
    with torch.no_grad():
        lt = orc.logsnr_schedule(torch.full((B,), 1.0), -5.1, 9.8)
        eref = orc.denoiser_forward(Qc.p, zt0.cpu(), lt, xemb.cpu())
    assert rel_l2(eps[0].cpu().numpy(), eref.numpy()) < 1e-5


def test_dropin_q_forward(gpu_device):
    """_netQ_U.forward keeps the reference contract: Q(x) and Q(x=None, b, device) -> (b, nz)."""
    from damc import synth
    from src import MCMC
    from src import diffusion_net as dn

    Q = dn._netQ_U(nc=3, nz=128, nxemb=64, ntemb=32, nif=8, diffusion_residual=True, n_interval=10,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
    synth.load_into(Q, 20)
    Q.to(gpu_device).eval()
    x = torch.rand(5, 3, 32, 32, device=gpu_device) * 2 - 1
    with torch.no_grad():
        z = Q(x)
        zp = Q(x=None, b=7, device=gpu_device)
    assert z.shape == (5, 128) and zp.shape == (7, 128)
    assert torch.isfinite(z).all() and torch.isfinite(zp).all()
    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=16, nc=3), 0).to(gpu_device)
    xs, zs = MCMC.gen_samples_with_diffusion_prior(b=6, device=gpu_device, netQ=Q, netG=G)
    assert xs.shape == (6, 3, 32, 32) and zs.shape == (6, 128)
