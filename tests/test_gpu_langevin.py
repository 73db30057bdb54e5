"""GPU parity: the HIP Langevin path (libdamc via damc.langevin / src.MCMC) vs the reference's
golden vectors and the oracle.

Tolerances (fp32; SURVEY.md §4, ~4x the reference's own fp32-vs-fp64 / thread-count spread):
  gradients rel-L2 <= 1e-5;  1 posterior step rel-L2(z) <= 1e-6;  10 no-noise steps <= 2e-4;
  30 steps (injected noise) <= 2e-3;  recon MSE rel <= 1e-5;  60 prior steps <= 1e-4.
"""
import numpy as np
import pytest
import torch

from conftest import G_NAMES, build_g_case, load_golden, rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lv(gpu_device):
    from damc import langevin

    return langevin


@pytest.mark.parametrize("name", G_NAMES)
def test_generator_forward(lv, gpu_device, name):
    c = build_g_case(name, gpu_device)
    xh = lv.generator_forward(c["z0"], c["G"]).cpu().numpy()
    if "gen_x" in c["rec"]:
        assert rel_l2(xh, c["rec"]["gen_x"]) < 1e-5
    else:
        assert rel_l2(xh[:, :, ::4, ::4], c["rec"]["gen_x_sub4"]) < 1e-5


@pytest.mark.parametrize("name", G_NAMES)
def test_likelihood_and_ebm_gradients(lv, gpu_device, name):
    c = build_g_case(name, gpu_device)
    g = lv.likelihood_grad(c["z0"], c["x"], c["G"], c["meta"]["sigma"]).cpu().numpy()
    assert rel_l2(g, c["rec"]["lik_grad0"]) < 1e-5
    e, ge = lv.ebm_energy_grad(c["z0"], c["E"])
    assert rel_l2(e.cpu().numpy(), c["rec"]["ebm_e"]) < 1e-5
    assert rel_l2(ge.cpu().numpy(), c["rec"]["ebm_grad0"]) < 1e-5


@pytest.mark.parametrize("name", G_NAMES)
def test_posterior_langevin_matches_reference(lv, gpu_device, name):
    c = build_g_case(name, gpu_device)
    m, rec = c["meta"], c["rec"]
    z = c["z0"].clone()
    lv.posterior_langevin(z, c["x"], c["G"], c["E"], 1, m["sigma"], m["step"], False)
    assert rel_l2(z.cpu().numpy(), rec["post_z1"]) < 1e-6
    z = c["z0"].clone()
    lv.posterior_langevin(z, c["x"], c["G"], c["E"], 10, m["sigma"], m["step"], False)
    assert rel_l2(z.cpu().numpy(), rec["post_z10"]) < 2e-4
    mse = ((lv.generator_forward(z, c["G"]) - c["x"]) ** 2).mean(dim=(1, 2, 3)).cpu().numpy()
    assert np.max(np.abs(mse - rec["recon_mse10"]) / rec["recon_mse10"]) < 1e-5
    z = c["z0"].clone()
    lv.posterior_langevin(z, c["x"], c["G"], c["E"], 30, m["sigma"], m["step"], True, noise=c["post_noise"])
    assert rel_l2(z.cpu().numpy(), rec["post_z30"]) < 2e-3


@pytest.mark.parametrize("engine", ["auto", "valu", "mfma"])
@pytest.mark.parametrize("name", ["cifar10_w16", "svhn_w16", "mnist_w16", "cifar10_full"])
def test_prior_langevin_matches_reference(lv, gpu_device, name, engine):
    c = build_g_case(name, gpu_device)
    if engine == "mfma" and c["zp0"].shape[1] % 16:
        pytest.skip("the MFMA prior engine needs nz % 16 == 0")
    z = c["zp0"].clone()
    lv.prior_langevin(z, c["E"], 5, c["meta"]["prior_step"], False, engine=engine)
    assert rel_l2(z.cpu().numpy(), c["rec"]["prior_z5"]) < 1e-6
    z = c["zp0"].clone()
    lv.prior_langevin(z, c["E"], 60, c["meta"]["prior_step"], True, noise=c["prior_noise"], engine=engine)
    assert rel_l2(z.cpu().numpy(), c["rec"]["prior_z60"]) < 1e-4


def test_prior_mfma_engine_large_batch(lv, gpu_device):
    """B = 2048 chains (past the MFMA engine's batch threshold): the 16-chain MFMA tiles against the fp64
    oracle (5 no-noise steps; a 2,048-row tail tile of 16 is exact), against the VALU engine (20 Philox steps:
    the same noise stream, so only summation order differs) and their step diagnostics."""
    from damc import synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    E = synth.load_into(dn._netE(nz=128), 10).to(gpu_device).eval()
    z0 = torch.from_numpy(synth.normal_f32(41, 0, (2050, 128))).to(gpu_device)  # 2050: a partial last tile
    ref = orc.prior_langevin(orc.ebm_params(E, torch.float64), z0.cpu().double(), 5, 0.4)
    z = z0.clone()
    lv.prior_langevin(z, E, 5, 0.4, False, engine="mfma")
    assert rel_l2(z.cpu().numpy(), ref.numpy()) < 1e-6
    za, zb = z0.clone(), z0.clone()
    da = lv.prior_langevin(za, E, 20, 0.4, True, seed=9, diag=True, engine="mfma")
    db = lv.prior_langevin(zb, E, 20, 0.4, True, seed=9, diag=True, engine="valu")
    assert rel_l2(za.cpu().numpy(), zb.cpu().numpy()) < 1e-5
    assert rel_l2(da.cpu().numpy(), db.cpu().numpy()) < 1e-5
    zc = z0.clone()
    lv.prior_langevin(zc, E, 20, 0.4, True, seed=9, engine="auto")  # 2050 >= the default threshold: MFMA
    assert torch.equal(zc, za)


def test_toy_posterior_matches_reference(lv, gpu_device):
    from damc import synth
    from damc.toy import ToyG

    rec, meta = load_golden("toy")
    G = synth.load_into(ToyG(), 0).to(gpu_device)
    B, nz = meta["B"], meta["nz"]
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, nz))).to(gpu_device)
    x = torch.from_numpy(rec["x"]).to(gpu_device)
    noise = torch.from_numpy(np.stack([synth.normal_f32(3, 100 + i, (B, nz))
                                       for i in range(meta["steps"])])).to(gpu_device)
    z = z0.clone()
    lv.posterior_langevin(z, x, G, None, 1, meta["sigma"], meta["step"], True, noise=noise)
    assert rel_l2(z.cpu().numpy(), rec["post_z1"]) < 1e-6
    z = z0.clone()
    lv.posterior_langevin(z, x, G, None, meta["steps"], meta["sigma"], meta["step"], True, noise=noise)
    assert rel_l2(z.cpu().numpy(), rec["post_z1000"]) < 2e-3


# ------------------------------------------------------------------ BASELINE-size checks
def _cifar_full(device, B):
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0).to(device).eval()
    E = synth.load_into(dn._netE(nz=128), 10).to(device).eval()
    x = torch.from_numpy(synth.uniform_f32(11, 0, (B, 3, 32, 32))).to(device)
    z0 = torch.from_numpy(synth.normal_f32(12, 0, (B, 128))).to(device)
    return G, E, x, z0


def test_cifar_b128_step_vs_oracle(lv, gpu_device):
    """BASELINE config (CIFAR-10, B=128, nz=128, ngf=128): one posterior step.

    A few rows of this batch have ill-conditioned likelihood gradients: the fp32 CPU
    restatement (= the reference's arithmetic) itself sits up to ~5e-4 from an fp64 evaluation
    there.  The criterion is therefore accuracy-relative: the HIP result's distance to fp64 must
    stay within 3x the fp32 reference arithmetic's distance to fp64 (+ a 1e-7 floor).
    """
    from oracle import damc_oracle as orc

    G, E, x, z0 = _cifar_full(gpu_device, 128)
    z = z0.clone()
    lv.posterior_langevin(z, x, G, E, 1, 0.1, 0.1, False)
    L32, P32 = orc.generator_layers(G), orc.ebm_params(E)
    L64, P64 = orc.generator_layers(G, torch.float64), orc.ebm_params(E, torch.float64)
    ref32 = orc.posterior_langevin(L32, P32, z0.cpu(), x.cpu(), 1, 0.1, 0.1).numpy()
    ref64 = orc.posterior_langevin(L64, P64, z0.cpu().double(), x.cpu().double(), 1, 0.1, 0.1).numpy()
    zg = z.cpu().numpy()
    assert rel_l2(zg, ref64) <= 3 * rel_l2(ref32, ref64) + 1e-7
    assert rel_l2(zg, ref32) < 2e-5
    g = lv.likelihood_grad(z0, x, G, 0.1).cpu().numpy()
    g32 = orc.likelihood_grad(L32, z0.cpu(), x.cpu(), 0.1)[0].numpy()
    g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 0.1)[0].numpy()
    assert rel_l2(g, g64) <= 3 * rel_l2(g32, g64) + 1e-6


def test_philox_noise_statistics(lv, gpu_device):
    n = lv.philox_normal(4, 512, 128, seed=1234, device=gpu_device).double().cpu().numpy().ravel()
    assert abs(n.mean()) < 5e-3 and abs(n.var() - 1.0) < 1e-2
    from scipy import stats

    assert stats.kstest(n[:200000], "norm").pvalue > 1e-3
    # different chains / steps / seeds are different streams
    a = lv.philox_normal(1, 2, 128, seed=1, device=gpu_device).cpu().numpy()
    assert np.abs(a[0, 0] - a[0, 1]).max() > 0.1
    b = lv.philox_normal(1, 2, 128, seed=2, device=gpu_device).cpu().numpy()
    assert np.abs(a - b).max() > 0.1
    # chain_base shifts the stream: chains [4, 8) of an 8-chain draw == a 4-chain draw at base 4
    full = lv.philox_normal(3, 8, 100, seed=9, device=gpu_device).cpu().numpy()
    part = lv.philox_normal(3, 4, 100, seed=9, device=gpu_device, chain_base=4).cpu().numpy()
    assert np.array_equal(full[:, 4:], part)


def test_sharded_chains_are_bitwise_identical(lv, gpu_device):
    """Noise keyed by GLOBAL chain index: 2 shards of 4 chains == 1 batch of 8, bit for bit."""
    G, E, x, z0 = _cifar_full(gpu_device, 8)
    za = z0.clone()
    lv.posterior_langevin(za, x, G, E, 5, 0.1, 0.1, True, seed=77)
    zb = [z0[:4].clone(), z0[4:].clone()]
    lv.posterior_langevin(zb[0], x[:4].contiguous(), G, E, 5, 0.1, 0.1, True, seed=77, chain_base=0)
    lv.posterior_langevin(zb[1], x[4:].contiguous(), G, E, 5, 0.1, 0.1, True, seed=77, chain_base=4)
    assert torch.equal(za, torch.cat(zb))
    pa = torch.cat([z0, z0]).contiguous()
    lv.prior_langevin(pa, E, 20, 0.4, True, seed=5)
    pb = [torch.cat([z0, z0])[:10].clone(), torch.cat([z0, z0])[10:].clone()]
    lv.prior_langevin(pb[0], E, 20, 0.4, True, seed=5, chain_base=0)
    lv.prior_langevin(pb[1], E, 20, 0.4, True, seed=5, chain_base=10)
    assert torch.equal(pa, torch.cat(pb))


def test_dropin_mcmc_api(gpu_device):
    """src.MCMC keeps the reference's call surface: in-place z, detach, requires_grad toggling."""
    from src import MCMC

    G, E, x, z0 = _cifar_full(gpu_device, 4)
    z = z0.clone().requires_grad_(True)
    out = MCMC.sample_langevin_post_z_with_prior(z=z, x=x, netG=G, netE=E, g_l_steps=3, g_llhd_sigma=0.1,
                                                 g_l_with_noise=True, g_l_step_size=0.1, verbose=True)
    assert out.data_ptr() == z.data_ptr() and not out.requires_grad
    assert not torch.equal(out, z0)
    assert all(p.requires_grad for p in G.parameters()) and all(p.requires_grad for p in E.parameters())
    zn = torch.cat([z0, torch.randn_like(z0, requires_grad=True)], dim=0)
    out = MCMC.sample_langevin_prior_z(z=zn, netE=E, e_l_steps=10, e_l_step_size=0.4, e_l_with_noise=True,
                                       verbose=True)
    assert out.shape == (8, 128) and torch.isfinite(out).all()
    xs = MCMC.gen_samples(bs=16, nz=128, netE=E, netG=G, e_l_steps=5, e_l_step_size=0.4, e_l_with_noise=True)
    assert xs.shape == (16, 3, 32, 32) and torch.isfinite(xs).all() and xs.abs().max() <= 1.0


def test_verbose_diagnostics_match_oracle(lv, gpu_device):
    """diag = {sum E, |G(z)-x|^2/(2s^2), |z|^2/2, mean grad} per step, as the reference logs them."""
    from oracle import damc_oracle as orc

    G, E, x, z0 = _cifar_full(gpu_device, 8)
    z = z0.clone()
    d = lv.posterior_langevin(z, x, G, E, 1, 0.1, 0.1, False, diag=True).cpu().numpy()[0]
    L, P = orc.generator_layers(G), orc.ebm_params(E)
    gl, lik, _ = orc.likelihood_grad(L, z0.cpu(), x.cpu(), 0.1)
    e, ge = orc.ebm_energy_grad(P, z0.cpu())
    want = [float(e.sum()), float(lik), float(0.5 * (z0.cpu() ** 2).sum()), float((gl + ge + z0.cpu()).mean())]
    assert np.allclose(d[:3], want[:3], rtol=1e-4, atol=1e-4)
    assert abs(d[3] - want[3]) < 1e-4 * max(1.0, abs(want[3]))


def test_kmajor_batch_chunking_is_bitwise(lv, gpu_device, tmp_path):
    """The K-major conv engine splits the batch when a gathered tensor would reach 2^31 bytes (the
    full-width CelebA-HQ dgrad at B=64 does).  A child process forced to ~3 MB chunks
    (DAMC_KM_CHUNK_BYTES) must reproduce the unchunked forward and gradient bit for bit."""
    import os
    import subprocess
    import sys

    from conftest import PKG, REPO

    G, E, x, z0 = _cifar_full(gpu_device, 8)
    g = lv.likelihood_grad(z0, x, G, 0.1).cpu().numpy()
    xh = lv.generator_forward(z0, G).cpu().numpy()
    out = str(tmp_path / "chunked.npz")
    code = (
        "import sys, numpy as np\n"
        f"sys.path[:0] = [{os.path.join(REPO, 'tests')!r}, {PKG!r}, {REPO!r}]\n"
        "import test_gpu_langevin as t\n"
        "from damc import langevin as lv\n"
        "G, E, x, z0 = t._cifar_full('cuda:0', 8)\n"
        f"np.savez({out!r}, g=lv.likelihood_grad(z0, x, G, 0.1).cpu().numpy(),"
        " xh=lv.generator_forward(z0, G).cpu().numpy())\n")
    env = dict(os.environ, DAMC_KM_CHUNK_BYTES=str(3 << 20))
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=600)
    r = np.load(out)
    assert np.array_equal(r["g"], g) and np.array_equal(r["xh"], xh)


def test_limb_engine_as_accurate_as_fp32_mfma(lv, gpu_device):
    """The limb engine (fp32 operands as 3 bf16 limbs, 6 limb products on bf16 MFMA, fp32 accumulate)
    against the fp32-MFMA engine, both measured against an fp64 evaluation of the same CIFAR-10
    full-width generator: the limb path must be as close to fp64 as exact fp32 arithmetic is
    (within 1.5x), on the likelihood gradient, the forward image and one posterior step."""
    from damc import _lib
    from oracle import damc_oracle as orc

    G, E, x, z0 = _cifar_full(gpu_device, 32)
    L64 = orc.generator_layers(G, torch.float64)
    P64 = orc.ebm_params(E, torch.float64)
    g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 0.1)[0].numpy()
    x64 = orc.generator_sample(L64, z0.cpu().double()).numpy()
    z64 = orc.posterior_langevin(L64, P64, z0.cpu().double(), x.cpu().double(), 1, 0.1, 0.1).numpy()

    def run():
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 1, 0.1, 0.1, False)
        return (lv.likelihood_grad(z0, x, G, 0.1).cpu().numpy(), lv.generator_forward(z0, G).cpu().numpy(),
                z.cpu().numpy())

    limb = run()
    with _lib.exact_fp32():
        exact = run()
    assert _lib.current_engine() == _lib.ENGINE_LIMB  # the context restored the default engine
    for got, ex, ref in zip(limb, exact, (g64, x64, z64)):
        e_limb, e_exact = rel_l2(got, ref), rel_l2(ex, ref)
        assert e_limb <= 1.5 * e_exact + 1e-7, (e_limb, e_exact)


def test_engine_is_per_call_not_global(lv, gpu_device):
    """The engine travels in each call's descriptor: a thread inside exact_fp32() and the main thread on the
    limb engine run at the same time without affecting each other, and each reproduces its own serial result."""
    import threading

    from damc import _lib

    G, E, x, z0 = _cifar_full(gpu_device, 8)
    limb = lv.likelihood_grad(z0, x, G, 0.1).cpu()
    with _lib.exact_fp32():
        exact = lv.likelihood_grad(z0, x, G, 0.1).cpu()
    assert not torch.equal(limb, exact)  # the two engines round differently
    out = {}

    def worker():
        with _lib.exact_fp32():
            for _ in range(4):
                out["exact"] = lv.likelihood_grad(z0, x, G, 0.1).cpu()

    t = threading.Thread(target=worker)
    t.start()
    for _ in range(4):
        out["limb"] = lv.likelihood_grad(z0, x, G, 0.1).cpu()
    t.join()
    assert torch.equal(out["limb"], limb) and torch.equal(out["exact"], exact)


def test_g_update_backward_runs_on_the_forward_engine(gpu_device):
    """x_hat = G(z) inside exact_fp32() with loss.backward() outside must give the exact engine's
    gradients (the backward uses the forward's recorded engine), not read buffers the forward never wrote."""
    from damc import _lib

    G, E, x, z0 = _cifar_full(gpu_device, 8)
    G.train()
    for p in G.parameters():
        p.requires_grad_(True)

    def grads(inside):
        G.zero_grad(set_to_none=True)
        if inside:
            with _lib.exact_fp32():
                xh = G(z0)
            loss = torch.sum((xh - x) ** 2, dim=[1, 2, 3]).mean()
        else:
            with _lib.exact_fp32():
                xh = G(z0)
                loss = torch.sum((xh - x) ** 2, dim=[1, 2, 3]).mean()
        loss.backward()  # outside the context when inside=True
        return [p.grad.detach().clone() for p in G.parameters()]

    split = grads(True)
    whole = grads(False)
    for a, b in zip(split, whole):
        assert torch.equal(a, b)


@pytest.mark.parametrize("net,B", [("cifar10", 4), ("cifar10", 16), ("svhn", 64), ("celeba64", 32), ("celebaHQ", 8)])
def test_split_k_is_bitwise_the_unsplit_kernel(lv, gpu_device, monkeypatch, net, B):
    """Split-K of the limb-engine convs at small batch (gemm.hip x3_ksplit: one sign block per slice, summed in the
    kernel's order and rounding) gives the same bits as the unsplit kernel: 3 posterior steps at full width with
    DAMC_X3_KSPLIT=0 vs the default -- F32A, register slabs, the reduce launch with the fused output-layer projection
    -- vs the two-kernel projection (DAMC_REDUCE_PROJ=0) and the round-6 in-GEMM ordered fix-up (DAMC_X3_FIXUP=1,
    opt-in: every slice of a tile combines one band of its rows once all slices have arrived, the last arriver takes
    any unclaimed band); and, at CIFAR, the opt-in 64 x 128 tile on the limb-gathering path (gemm.hip X3_NARROW,
    DAMC_X3_NARROW=1 with DAMC_X3_F32A=0) against all of them.  Per-rank batches of the BASELINE configs: CIFAR B=16
    (8-way headline), SVHN B=64, CelebA-64 B=32, CelebA-HQ B=8."""
    from damc import synth
    from src import diffusion_net as dn

    ctor, nz, hw, ngf, sigma = {"cifar10": ("_netG_cifar10", 128, 32, 128, 0.1), "svhn": ("_netG_svhn", 100, 32, 64, 0.1),
                                "celeba64": ("_netG_celeba64", 100, 64, 128, 0.1),
                                "celebaHQ": ("_netG_celebaHQ", 128, 256, 128, 1.0)}[net]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(gpu_device).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, hw, hw))).to(gpu_device)
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, nz))).to(gpu_device)
    out = {}
    modes = [("unsplit", "0", "0", "0", "1"), ("split", "1", "0", "0", "1"), ("fixup", "1", "0", "1", "1"),
             ("reduce2", "1", "0", "0", "0")]
    if net == "cifar10":
        modes.append(("narrow", "1", "1", "1", "1"))
    for mode, split, narrow, fixup, rproj in modes:
        # reduce2: the reduce and the output-layer projection as two kernels (DAMC_REDUCE_PROJ=0) instead of the fused
        # x3_ksplit_reduce_proj_kernel
        monkeypatch.setenv("DAMC_X3_FIXUP", fixup)
        monkeypatch.setenv("DAMC_REDUCE_PROJ", rproj)
        monkeypatch.setenv("DAMC_X3_KSPLIT", split)
        monkeypatch.setenv("DAMC_X3_NARROW", narrow)
        monkeypatch.setenv("DAMC_X3_F32A", "0" if narrow == "1" else "1")  # the 64 x 128 tile gathers limbs
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 3, sigma, 0.1, True, seed=77)
        torch.cuda.synchronize()
        out[mode] = z.cpu()
    assert torch.isfinite(out["split"]).all() and not torch.equal(out["split"], z0.cpu())
    for mode in out:
        assert torch.equal(out["unsplit"], out[mode]), mode


@pytest.mark.parametrize("net,B", [("cifar10", 5), ("cifar10", 128), ("celeba64", 4)])
def test_lds_staged_output_projection_is_bitwise_the_direct_kernel(lv, gpu_device, monkeypatch, net, B):
    """The output layer's projection stage staged through LDS (generator.hip smallc_proj_lds_kernel: same MFMA
    sequence, operands from LDS) gives the same bits as the direct-load kernel: 2 posterior steps at full width
    (CIFAR k3: one 32-column tile, ragged last wave at B=5; CelebA-64 k4 s2: two tiles) with
    DAMC_SMALLC_PROJ_LDS=0 vs 1 (with the round-4 proj16 kernel and the fused projection switched off, so these two
    kernels are the ones compared)."""
    from damc import synth
    from src import diffusion_net as dn

    nz, hw = (128, 32) if net == "cifar10" else (100, 64)
    G = synth.load_into(getattr(dn, "_netG_" + net)(nz=nz, ngf=128, nc=3), 0).to(gpu_device).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, hw, hw))).to(gpu_device)
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, nz))).to(gpu_device)
    out = {}
    monkeypatch.setenv("DAMC_SMALLC_PROJ16", "0")
    monkeypatch.setenv("DAMC_SMALLC_FUSE", "0")
    for mode in ("0", "1"):
        monkeypatch.setenv("DAMC_SMALLC_PROJ_LDS", mode)
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 2, 0.1, 0.1, True, seed=78)
        torch.cuda.synchronize()
        out[mode] = z.cpu()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])


@pytest.mark.parametrize("B", [16, 37])
def test_fused_posterior_update_is_bitwise(lv, gpu_device, monkeypatch, B):
    """The posterior update kernel sums the first layer's split-K slabs itself (slab_sum4's fixed order) and writes z's
    limbs for the next step's first layer: 3 noisy steps bitwise equal to the separate slab-sum and limb-split
    kernels (DAMC_POST_FUSE=0)."""
    G, E, x, z0 = _cifar_full(gpu_device, B)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DAMC_POST_FUSE", mode)
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 3, 0.1, 0.1, True, seed=77)
        torch.cuda.synchronize()
        out[mode] = z.cpu()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])


@pytest.mark.parametrize("name,B", [("cifar10", 16), ("cifar10", 128), ("svhn", 64), ("celeba64", 32)])
def test_f32a_posterior_is_bitwise(lv, gpu_device, monkeypatch, name, B):
    """DAMC_X3_F32A=1: the limb-engine convolutions gather fp32 activations / gradients and split them into limbs in
    registers (gemm.hip X3_F32A), the output layer's dgrad writes fp32: 2 noisy posterior steps bitwise equal to the
    limb-gathering path (B=16 runs split-K with register slabs, B=128 unsplit)."""
    from damc import synth
    from src import diffusion_net as dn

    ctor, nz, ngf, hw = {"cifar10": ("_netG_cifar10", 128, 128, 32), "svhn": ("_netG_svhn", 100, 64, 32),
                         "celeba64": ("_netG_celeba64", 100, 128, 64)}[name]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(gpu_device).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(11, 0, (B, 3, hw, hw))).to(gpu_device)
    z0 = torch.from_numpy(synth.normal_f32(12, 0, (B, nz))).to(gpu_device)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DAMC_X3_F32A", mode)
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 2, 0.1, 0.1, True, seed=5)
        torch.cuda.synchronize()
        out[mode] = z.cpu()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])


@pytest.mark.parametrize("B,f32a", [(16, "1"), (128, "1"), (16, "0"), (128, "0")])
def test_fused_output_projection_is_bitwise(lv, gpu_device, monkeypatch, B, f32a):
    """The last ConvT's epilogue runs the output layer's per-tap projection (gemm.hip GemmArgs::proj_out; B=16
    splits K, so there the projection runs as proj_rows_kernel over the reduce's output): 2 noisy posterior steps
    bitwise equal to the separate projection kernel (DAMC_SMALLC_FUSE=0), which shares proj16's arithmetic and its
    128-channel chunks.  Both tiles: the F32A kernel (each 128-channel N tile projects its chunk) and the
    limb-gathering 128 x 256 layout (DAMC_X3_F32A=0, every channel in one tile)."""
    G, E, x, z0 = _cifar_full(gpu_device, B)
    monkeypatch.setenv("DAMC_X3_F32A", f32a)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DAMC_SMALLC_FUSE", mode)
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 2, 0.1, 0.1, True, seed=9)
        torch.cuda.synchronize()
        out[mode] = z.cpu()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])


@pytest.mark.parametrize("B", [8, 16, 32, 48, 64, 128])
def test_skinny_first_layer_is_bitwise(lv, gpu_device, monkeypatch, B):
    """The first layer at per-rank batches (B <= 32): z . W on gemm.hip's x3_skinny_kernel and its input gradient's
    split-K slabs on km_skinny_kernel (fragments straight into registers; up to B = 64 as 32-row workgroups, round
    6, or as two 32-row tiles per wave, DAMC_KM_SKINNY_MT=2, round 5): 2 noisy posterior steps bitwise equal to
    the tiled kernels (DAMC_X3_SKINNY=0, DAMC_KM_SKINNY=0), with the skinny kernel reading the weights as fp32 rows
    split in registers (round 5, default) and as the packed limbs (DAMC_X3_SKINNY_F32B=0)."""
    G, E, x, z0 = _cifar_full(gpu_device, B)
    out = {}
    for mode, f32b, mt in (("0", "1", "1"), ("1", "1", "1"), ("1", "0", "1"), ("1", "1", "2")):
        monkeypatch.setenv("DAMC_X3_SKINNY", mode)
        monkeypatch.setenv("DAMC_KM_SKINNY", mode)
        monkeypatch.setenv("DAMC_X3_SKINNY_F32B", f32b)
        monkeypatch.setenv("DAMC_KM_SKINNY_MT", mt)
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 2, 0.1, 0.1, True, seed=13)
        torch.cuda.synchronize()
        out[mode + f32b + mt] = z.cpu()
    assert torch.isfinite(out["111"]).all()
    assert torch.equal(out["011"], out["111"])
    assert torch.equal(out["011"], out["101"])
    assert torch.equal(out["011"], out["112"])


@pytest.mark.parametrize("net,B", [("cifar10", 100), ("cifar10", 128), ("celeba64", 32)])
def test_lds_staged_gather_is_bitwise_the_direct_gather(lv, gpu_device, monkeypatch, net, B):
    """The output layer's gather (delta, x_hat from the per-tap projections and their 128-channel partials)
    staged through LDS (generator.hip smallc_gather_lds_kernel for k3 s1 row strips, smallc_gather_s2_lds_kernel for
    k4 s2 16 x 32 tiles): 2 noisy posterior steps bitwise equal to the direct per-pixel gather
    (DAMC_SMALLC_GATHER_LDS=0), at batches whose tiles fill the chip (the LDS forms run from 256 workgroups)."""
    from damc import synth
    from src import diffusion_net as dn

    nz, hw = (128, 32) if net == "cifar10" else (100, 64)
    G = synth.load_into(getattr(dn, "_netG_" + net)(nz=nz, ngf=128, nc=3), 0).to(gpu_device).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, hw, hw))).to(gpu_device)
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, nz))).to(gpu_device)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DAMC_SMALLC_GATHER_LDS", mode)
        z = z0.clone()
        lv.posterior_langevin(z, x, G, E, 2, 0.1, 0.1, True, seed=21)
        torch.cuda.synchronize()
        out[mode] = z.cpu()
    assert torch.isfinite(out["1"]).all()
    assert torch.equal(out["0"], out["1"])


def test_spectral_norm_nets_in_eval_mode(lv, gpu_device):
    """use_spc_norm=True generators and e_sn=True EBMs (nn.utils.spectral_norm, diffusion_net.py:8-16, 21-44, 208-210)
    on the HIP path in eval mode, the mode of the reference's Langevin chains (train_gen_recon.py:191-193): after a few
    train-mode forwards have moved u and v, the posterior chain (10 no-noise steps) and the prior chain match the
    oracle on the weights the layers' own forward pre-hooks compute (train mode: the next test)."""
    from damc import synth
    from damc import training
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=16, nc=3, use_spc_norm=True), 4).to(gpu_device)
    E = synth.load_into(dn._netE(nz=128, e_sn=True), 5).to(gpu_device)
    z0 = torch.from_numpy(synth.normal_f32(91, 0, (8, 128))).to(gpu_device)
    x = torch.from_numpy(synth.uniform_f32(91, 1, (8, 3, 32, 32))).to(gpu_device)
    with training.stock_pytorch(), torch.no_grad():
        for _ in range(3):  # power iterations move u, v away from their initial values
            G.train()(z0)
            E.train()(z0)
    G.eval()
    E.eval()
    z = z0.clone()
    lv.posterior_langevin(z, x, G, E, 10, 0.3, 0.1, False)
    with training.stock_pytorch(), torch.no_grad():
        G(z0)  # the hooks set every layer's weight (eval: no power iteration)
        E(z0)
    L, P = orc.generator_layers(G), orc.ebm_params(E)
    ref = orc.posterior_langevin(L, P, z0.cpu(), x.cpu(), 10, 0.3, 0.1)
    assert rel_l2(z.cpu().numpy(), ref.numpy()) < 2e-4
    zp = torch.cat([z0, z0]).contiguous()
    lv.prior_langevin(zp, E, 5, 0.4, False)
    refp = orc.prior_langevin(P, torch.cat([z0, z0]).cpu(), 5, 0.4)
    assert rel_l2(zp.cpu().numpy(), refp.numpy()) < 1e-5


def _sn_buffers(net):
    return [t for n, t in net.named_buffers() if n.endswith("weight_u") or n.endswith("weight_v")]


def test_spectral_norm_nets_in_train_mode(lv, gpu_device):
    """Spectral-norm G and E in train mode (nn.utils.spectral_norm, diffusion_net.py:8-16, 21-44, 208-210): every
    forward of the reference advances u and v by one power iteration, so the weights move from step to step (fresh u:
    sigma still converging).  The HIP chains run one step per call after that step's power iterations: against the
    reference's own loops (MCMC.py:27-46, 48-74) on deep copies of the stock modules with the same injected noise, z
    matches (fp32: rel-L2 <= 2e-4 over 6 posterior steps, <= 1e-5 over 5 prior steps) and every u, v buffer is bitwise
    the reference's afterwards; likelihood_grad / generator_forward / ebm_energy_grad each advance once, as one forward."""
    import copy

    from damc import synth
    from damc import training
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=16, nc=3, use_spc_norm=True), 4).to(gpu_device).train()
    E = synth.load_into(dn._netE(nz=128, e_sn=True), 5).to(gpu_device).train()
    G2, E2 = copy.deepcopy(G), copy.deepcopy(E)
    z0 = torch.from_numpy(synth.normal_f32(93, 0, (8, 128))).to(gpu_device)
    x = torch.from_numpy(synth.uniform_f32(93, 1, (8, 3, 32, 32))).to(gpu_device)
    noise = torch.from_numpy(synth.normal_f32(93, 2, (6, 8, 128))).to(gpu_device)
    sigma, step = 0.3, 0.1
    z = z0.clone()
    lv.posterior_langevin(z, x, G, E, 6, sigma, step, True, noise=noise)
    zr = z0.clone().requires_grad_(True)
    with training.stock_pytorch():
        for i in range(6):
            lk = 1.0 / (2.0 * sigma * sigma) * torch.sum((G2(zr) - x) ** 2)
            total = lk + E2(zr).sum() + 0.5 * torch.sum(zr ** 2)
            g = torch.autograd.grad(total, zr)[0]
            zr.data = zr.data - 0.5 * step * step * g + step * noise[i]
    assert rel_l2(z.cpu().numpy(), zr.detach().cpu().numpy()) < 2e-4
    for a, b in zip(_sn_buffers(G) + _sn_buffers(E), _sn_buffers(G2) + _sn_buffers(E2)):
        assert torch.equal(a, b)
    # a chain whose weights did not move would be far off: the stepping is what the match rests on
    zf = z0.clone()
    G3, E3 = copy.deepcopy(G).eval(), copy.deepcopy(E).eval()
    lv.posterior_langevin(zf, x, G3, E3, 6, sigma, step, True, noise=noise)
    assert rel_l2(zf.cpu().numpy(), zr.detach().cpu().numpy()) > 10 * rel_l2(z.cpu().numpy(), zr.detach().cpu().numpy())

    zp = torch.cat([z0, z0]).contiguous()
    pn = torch.from_numpy(synth.normal_f32(93, 3, (5, 16, 128))).to(gpu_device)
    lv.prior_langevin(zp, E, 5, 0.4, True, noise=pn)
    zq = torch.cat([z0, z0]).requires_grad_(True)
    with training.stock_pytorch():
        for i in range(5):
            g = torch.autograd.grad(E2(zq).sum() + 0.5 * torch.sum(zq ** 2), zq)[0]
            zq.data = zq.data - 0.5 * 0.4 * 0.4 * g + 0.4 * pn[i]
    assert rel_l2(zp.cpu().numpy(), zq.detach().cpu().numpy()) < 1e-5
    for a, b in zip(_sn_buffers(E), _sn_buffers(E2)):
        assert torch.equal(a, b)

    xh = lv.generator_forward(z0, G)
    lv.ebm_energy_grad(z0, E)
    with training.stock_pytorch(), torch.no_grad():
        xr = G2(z0)
        E2(z0)
    assert rel_l2(xh.cpu().numpy(), xr.cpu().numpy()) < 1e-5
    for a, b in zip(_sn_buffers(G) + _sn_buffers(E), _sn_buffers(G2) + _sn_buffers(E2)):
        assert torch.equal(a, b)


def test_chain_cut_into_single_steps_is_bitwise(lv, gpu_device):
    """The stepping that train-mode spectral norm uses: a chain run as one call equals the same chain run one step per
    call (step_offset = i keys the in-kernel Philox), bitwise, for the posterior and the prior."""
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=32, nc=3), 4).to(gpu_device).eval()
    E = synth.load_into(dn._netE(nz=128), 5).to(gpu_device).eval()
    z0 = torch.from_numpy(synth.normal_f32(94, 0, (16, 128))).to(gpu_device)
    x = torch.from_numpy(synth.uniform_f32(94, 1, (16, 3, 32, 32))).to(gpu_device)
    z1, z2 = z0.clone(), z0.clone()
    lv.posterior_langevin(z1, x, G, E, 5, 0.3, 0.1, True, seed=77)
    for i in range(5):
        lv.posterior_langevin(z2, x, G, E, 1, 0.3, 0.1, True, seed=77, step_offset=i)
    assert torch.equal(z1, z2)
    p1, p2 = torch.cat([z0, z0]).contiguous(), torch.cat([z0, z0]).contiguous()
    lv.prior_langevin(p1, E, 5, 0.4, True, seed=78)
    for i in range(5):
        lv.prior_langevin(p2, E, 1, 0.4, True, seed=78, step_offset=i)
    assert torch.equal(p1, p2)
