"""GPU: the BASELINE configs beyond CIFAR-10 at their full widths and per-rank sizes on the HIP path
(BASELINE.json configs 2, 4, 5; workspace/src/diffusion_net.py:53-170 generators, :268-372 encoders,
workspace/train_gen_recon.py:64-92 their nz / ngf / nif):
  * SVHN _netG_svhn(nz=100, ngf=64), B=64: one step, and 30 steps with injected noise;
  * CelebA-64 _netG_celeba64(nz=100, ngf=128): B=32 (per rank of 256 over 8 GPUs) one step and 10 no-noise steps
    (the eval path) with the reconstruction MSE; B=256 (the whole batch on one GPU) one step;
  * CelebA-HQ _netG_celebaHQ(nz=128, ngf=128), sigma=1.0: B=8 (per rank of 64) one step; B=64 the likelihood
    gradient of the whole batch in one call;
  * Encoder_celeba64 / Encoder_celebaHQ at nif=64 (nemb 1024), and CelebA-HQ's Q(x): encoder + the 100-step
    reverse sweep (nxemb 1024, ntemb 128, injected noise) at B=8.
The criterion is accuracy-relative against an fp64 evaluation of the same algorithm (oracle/damc_oracle.py):
the HIP result's distance to fp64 must stay within 3x the fp32 oracle's (the reference's own arithmetic), plus
a small floor — per sample (median and 90th percentile) for latents and gradients, whose batches can hold a
sample sitting on a LeakyReLU kink; each test prints both distances."""
import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu

GEN = {  # name: (constructor, nz, ngf, image size)
    "cifar10": ("_netG_cifar10", 128, 128, 32),
    "svhn": ("_netG_svhn", 100, 64, 32),
    "celeba64": ("_netG_celeba64", 100, 128, 64),
    "celebaHQ": ("_netG_celebaHQ", 128, 128, 256),
}


def _case(name, B, device):
    from damc import synth
    from src import diffusion_net as dn

    ctor, nz, ngf, hw = GEN[name]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(device).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(device).eval()
    x = torch.from_numpy(synth.uniform_f32(11, 0, (B, 3, hw, hw))).to(device)
    z0 = torch.from_numpy(synth.normal_f32(12, 0, (B, nz))).to(device)
    return G, E, x, z0


def _oracles(G, E):
    from oracle import damc_oracle as orc

    return ((orc.generator_layers(G), orc.ebm_params(E)),
            (orc.generator_layers(G, torch.float64), orc.ebm_params(E, torch.float64)))


def _kink_rows(L64, z, rel=1e-6):
    """Samples with a hidden pre-activation within rel x its layer's RMS of the LeakyReLU kink (fp64 forward at z):
    their derivative (1 vs 0.2) is decided by rounding in any fp32 evaluation."""
    from oracle import damc_oracle as orc

    hs = orc.generator_forward(L64, z.double())
    kink = np.zeros(z.shape[0], dtype=bool)
    for h in hs[:-1]:
        a = h.abs().reshape(h.shape[0], -1)
        kink |= (a.min(dim=1).values < rel * h.pow(2).mean().sqrt()).numpy()
    return kink


def _kink_flip_bound(L64, P64, z0, x, sigma, step, rows, rel=1e-6):
    """Per kink sample: how far its one-step z can legitimately sit from the fp64 one.  A hidden unit within
    rel x its layer's RMS of the LeakyReLU kink may take the other derivative (1 vs 0.2) in any fp32 evaluation;
    for each such unit the fp64 step is recomputed with that unit's mask flipped (its activation negated, which
    flips the backward's sign test only), and the row's bound is the sum over its units of
    |z_flipped - z64| / |z64| (a triangle bound over any subset of flips)."""
    from oracle import damc_oracle as orc

    z0, x = z0.double(), x.double()
    hs_all = orc.generator_forward(L64, z0)
    rms = [h.pow(2).mean().sqrt() for h in hs_all[:-1]]
    c = 0.5 * step * step
    out = np.zeros(z0.shape[0])
    for r in np.nonzero(rows)[0]:
        zr, xr = z0[r:r + 1], x[r:r + 1]
        hs = orc.generator_forward(L64, zr)
        xh = hs[-1]
        delta = ((xh - xr) / (sigma * sigma)) * orc._act_grad_from_out(xh, L64[-1]["act"])
        g0 = orc.generator_vjp(L64, hs, delta)
        zref = zr - c * (g0 + zr + orc.ebm_energy_grad(P64, zr)[1])
        tot = 0.0
        for li, h in enumerate(hs[:-1]):
            for idx in torch.nonzero(h.abs() < rel * rms[li]):
                h2 = h.clone()
                v = h2[tuple(idx)]
                h2[tuple(idx)] = -v if v != 0 else -1e-30
                g2 = orc.generator_vjp(L64, hs[:li] + [h2] + hs[li + 1:], delta)
                tot += float((c * (g2 - g0)).norm() / zref.norm())
        out[r] = tot
    return out


def _check(what, got, ref32, ref64, floor, per_row=False, factor=3.0, kink=None, kink_bound=None):
    """Distance to fp64 against the fp32 reference arithmetic's.  per_row: per-sample relative errors, judged by
    their median and 90th percentile, and every row that is not a kink sample by the largest fp32-reference row
    error: a sample with a hidden pre-activation within fp32 rounding of the LeakyReLU kink can take the other
    derivative (1 vs 0.2) under any summation order (the SVHN B=64 batch's sample 54 has a first-layer unit at
    1.2e-8).  A kink row is held to the non-kink bound plus the effect of flipping its kink units' derivatives,
    computed in fp64 (_kink_flip_bound), with 1.5x slack for second-order terms between flips."""
    if not per_row:
        e_hip, e_32 = rel_l2(got, ref64), rel_l2(ref32, ref64)
        print("%s: |hip-fp64| %.2e  |fp32 reference arithmetic-fp64| %.2e" % (what, e_hip, e_32))
        assert e_hip <= factor * e_32 + floor, (what, e_hip, e_32)
        return
    rows = lambda a: np.array([rel_l2(a[i], ref64[i]) for i in range(ref64.shape[0])])  # noqa: E731
    eh, e3 = rows(got), rows(ref32)
    q = lambda e, p: float(np.quantile(e, p))  # noqa: E731
    print("%s: per-row |hip-fp64| median %.2e p90 %.2e max %.2e (row %d);  fp32 reference median %.2e p90 %.2e max %.2e"
          % (what, q(eh, .5), q(eh, .9), eh.max(), eh.argmax(), q(e3, .5), q(e3, .9), e3.max()))
    assert q(eh, .5) <= factor * q(e3, .5) + floor, what
    assert q(eh, .9) <= factor * q(e3, .9) + floor, what
    if kink is None:  # no kink analysis (the whole-batch gradient below): the ill-conditioned rows are only bounded
        assert eh.max() < 5e-2, what
        return
    if not kink.any():
        assert eh.max() <= factor * e3.max() + floor, what
        return
    if (~kink).any():
        print("%s: %d kink sample(s); the other rows' max |hip-fp64| %.2e vs the fp32 reference's %.2e"
              % (what, int(kink.sum()), eh[~kink].max(), e3[~kink].max()))
        base = factor * e3[~kink].max() + floor
        assert eh[~kink].max() <= base, what
    else:  # every sample has a near-kink unit (CelebA-HQ's 5.8M hidden units per sample): the median row's bound
        base = factor * q(e3, .5) + floor
    for r in np.nonzero(kink)[0]:
        print("%s: kink row %d |hip-fp64| %.2e  fp32 reference %.2e  flip bound %.2e"
              % (what, r, eh[r], e3[r], kink_bound[r]))
        assert eh[r] <= base + 1.5 * kink_bound[r], (what, r)


@pytest.mark.parametrize("name,B,steps,noise,sigma", [
    ("cifar10", 128, 1, False, 0.1), ("cifar10", 128, 10, False, 0.1),
    ("svhn", 64, 1, False, 0.1), ("svhn", 64, 30, True, 0.1),
    ("celeba64", 32, 1, False, 0.1), ("celeba64", 32, 10, False, 0.1), ("celeba64", 256, 1, False, 0.1),
    ("celebaHQ", 8, 1, False, 1.0)])
def test_full_width_posterior_vs_fp64(gpu_device, name, B, steps, noise, sigma):
    from damc import langevin as lv
    from oracle import damc_oracle as orc

    G, E, x, z0 = _case(name, B, gpu_device)
    (L32, P32), (L64, P64) = _oracles(G, E)
    nz = z0.shape[1]
    xi = torch.from_numpy(np.random.default_rng(B + steps).standard_normal((steps, B, nz)).astype(np.float32)) \
        if noise else None
    z = z0.clone()
    lv.posterior_langevin(z, x, G, E, steps, sigma, 0.1, noise, noise=None if xi is None else xi.to(gpu_device))
    zc, xc = z0.cpu(), x.cpu()
    r32 = orc.posterior_langevin(L32, P32, zc, xc, steps, sigma, 0.1, noise=xi).numpy()
    r64 = orc.posterior_langevin(L64, P64, zc.double(), xc.double(), steps, sigma, 0.1,
                                 noise=None if xi is None else xi.double()).numpy()
    # one step: per sample (a kink sample is bounded, not compared); several steps: the whole batch, whose rel-L2
    # both implementations grow chaotically
    kink = _kink_rows(L64, zc) if steps == 1 else None
    kb = _kink_flip_bound(L64, P64, zc, xc, sigma, 0.1, kink) if steps == 1 else None
    _check("%s B=%d %d step(s) z" % (name, B, steps), z.cpu().numpy(), r32, r64, 1e-7 if steps == 1 else 1e-6,
           per_row=steps == 1, kink=kink, kink_bound=kb)
    if steps == 10:  # eval path: reconstruction MSE of the 10-step no-noise posterior (eval_gen_recon.py:184-194)
        mse = ((lv.generator_forward(z, G) - x) ** 2).mean(dim=(1, 2, 3)).cpu().numpy()
        m32 = ((orc.generator_sample(L32, torch.from_numpy(r32)) - xc) ** 2).mean(dim=(1, 2, 3)).numpy()
        m64 = ((orc.generator_sample(L64, torch.from_numpy(r64)) - xc.double()) ** 2).mean(dim=(1, 2, 3)).numpy()
        _check("%s B=%d recon MSE" % (name, B), mse, m32, m64, 1e-7)


@pytest.mark.timeout(900)
def test_headline_posterior_30_noisy_steps_vs_fp64(gpu_device):
    """The bench's own posterior leg (BASELINE config 3: CIFAR-10 _netG_cifar10 ngf=128, nz=128, B=128, 30 steps,
    sigma 0.1, step 0.1; MCMC.py:48-74, train_gen_recon.py:203-205) with injected noise, the whole batch against
    fp64, accuracy-relative like the 10-step case (both fp32 implementations drift chaotically from fp64 over 30
    steps: the criterion is that the HIP arithmetic drifts no more than 3x the reference's own)."""
    from damc import langevin as lv
    from oracle import damc_oracle as orc

    B, steps = 128, 30
    G, E, x, z0 = _case("cifar10", B, gpu_device)
    (L32, P32), (L64, P64) = _oracles(G, E)
    xi = torch.from_numpy(np.random.default_rng(B + steps).standard_normal((steps, B, 128)).astype(np.float32))
    z = z0.clone()
    lv.posterior_langevin(z, x, G, E, steps, 0.1, 0.1, True, noise=xi.to(gpu_device))
    zc, xc = z0.cpu(), x.cpu()
    r32 = orc.posterior_langevin(L32, P32, zc, xc, steps, 0.1, 0.1, noise=xi).numpy()
    r64 = orc.posterior_langevin(L64, P64, zc.double(), xc.double(), steps, 0.1, 0.1, noise=xi.double()).numpy()
    _check("cifar10 B=128 30 noisy steps z", z.cpu().numpy(), r32, r64, 1e-6)
    # per sample: the median and 90th percentile rows against the fp32 reference's (no per-row max: a sample whose
    # trajectory crossed a LeakyReLU kink in either fp32 evaluation diverges chaotically in both)
    _check("cifar10 B=128 30 noisy steps z (per chain)", z.cpu().numpy(), r32, r64, 1e-6, per_row=True)


def test_headline_in_kernel_philox_equals_materialised_stream(gpu_device):
    """The bench's posterior leg with the in-kernel Philox4x32-10 draw (CIFAR-10 ngf=128, B=128, 30 steps, with_noise)
    is bitwise the same call fed damc_philox_normal's materialised posterior stream (same seed, steps 0..29, chains
    0..127) as injected noise: the in-kernel noise the bench times is exactly the stream the statistical tests check
    (test_philox_noise_statistics) and that the injected-noise parity tests stand in for."""
    from damc import langevin as lv

    B, steps, seed = 128, 30, 0x5EED1234
    G, E, x, z0 = _case("cifar10", B, gpu_device)
    za, zb = z0.clone(), z0.clone()
    lv.posterior_langevin(za, x, G, E, steps, 0.1, 0.1, True, seed=seed)
    xi = lv.philox_normal(steps, B, 128, seed, gpu_device)
    lv.posterior_langevin(zb, x, G, E, steps, 0.1, 0.1, True, noise=xi)
    torch.cuda.synchronize()
    assert torch.isfinite(za).all() and not torch.equal(za, z0)
    assert torch.equal(za, zb), float((za - zb).abs().max())
    # and the sharded form (chain_base) draws the same stream: the upper half alone, keyed by its global index
    zc = z0[64:].clone()
    lv.posterior_langevin(zc, x[64:].contiguous(), G, E, steps, 0.1, 0.1, True, seed=seed, chain_base=64)
    assert torch.equal(zc, za[64:])


@pytest.mark.parametrize("name,B,part", [("cifar10", 2752, 128), ("celebaHQ", 344, 8)])
def test_output_layer_dgrad_beyond_2gb_is_chunked(gpu_device, name, B, part):
    """Batches whose output-layer input gradient reaches 2^31 bytes (CIFAR's k3 layer from B = 2731 with fp32 out,
    CelebA-HQ's k4 s2 layer from B = 342 with limbs out) take a full posterior step: the limb-engine dgrad runs in
    per-sample chunks, and the first and last chains are bitwise the same chains run as a small batch
    (chain_base keys the noise by global index)."""
    from damc import langevin as lv

    G, E, x, z0 = _case(name, B, gpu_device)
    sigma = 1.0 if name == "celebaHQ" else 0.1
    za = z0.clone()
    lv.posterior_langevin(za, x, G, E, 1, sigma, 0.1, True, seed=77)
    assert torch.isfinite(za).all()
    for s in (0, B - part):
        zb = z0[s:s + part].clone()
        lv.posterior_langevin(zb, x[s:s + part].contiguous(), G, E, 1, sigma, 0.1, True, seed=77, chain_base=s)
        assert torch.equal(za[s:s + part], zb), (s, float((za[s:s + part] - zb).abs().max()))


def test_cifar_prior_60_steps_vs_fp64(gpu_device):
    """BASELINE headline's prior chain: 60 noisy steps (step 0.4, injected noise) on 2B = 256 chains of _netE(nz=128)
    (MCMC.py:27-46, train_gen_recon.py:207-209), whole batch against fp64, accuracy-relative."""
    from damc import langevin as lv
    from damc import synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    E = synth.load_into(dn._netE(nz=128), 10).to(gpu_device).eval()
    z0 = torch.from_numpy(synth.normal_f32(13, 0, (256, 128)))
    xi = torch.from_numpy(np.random.default_rng(60).standard_normal((60, 256, 128)).astype(np.float32))
    z = z0.to(gpu_device)
    lv.prior_langevin(z, E, 60, 0.4, True, noise=xi.to(gpu_device))
    r32 = orc.prior_langevin(orc.ebm_params(E), z0, 60, 0.4, noise=xi).numpy()
    r64 = orc.prior_langevin(orc.ebm_params(E, torch.float64), z0.double(), 60, 0.4, noise=xi.double()).numpy()
    _check("cifar prior 2B=256 60 steps z", z.cpu().numpy(), r32, r64, 1e-7)
    _check("cifar prior 2B=256 60 steps z (per chain)", z.cpu().numpy(), r32, r64, 1e-7, per_row=True,
           kink=np.zeros(256, dtype=bool))


def test_celebaHQ_b64_likelihood_gradient_vs_fp64(gpu_device):
    """CelebA-HQ's whole B=64 batch (BASELINE config 5 on one GPU) in one call: forward + input gradient."""
    from damc import langevin as lv
    from oracle import damc_oracle as orc

    G, E, x, z0 = _case("celebaHQ", 64, gpu_device)
    (L32, _), (L64, _) = _oracles(G, E)
    g = lv.likelihood_grad(z0, x, G, 1.0).cpu().numpy()
    g32 = orc.likelihood_grad(L32, z0.cpu(), x.cpu(), 1.0)[0].numpy()
    g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 1.0)[0].numpy()
    # 7 layers, 5 of them k4 s2 p1 with K = 16 Cout up to 16384, then the first layer's 32768-term sum: a bias in
    # the GEMM's rounding survives that sum where noise cancels, so this is the test of the limb engine's blocked,
    # sign-alternating accumulation (gemm.hip; without it the HIP median was 13x the fp32 reference's)
    _check("celebaHQ B=64 likelihood gradient", g, g32, g64, 1e-7, per_row=True)
    xh = lv.generator_forward(z0, G).cpu().numpy()
    _check("celebaHQ B=64 G(z)", xh, orc.generator_sample(L32, z0.cpu()).numpy(),
           orc.generator_sample(L64, z0.cpu().double()).numpy(), 1e-7)


@pytest.mark.parametrize("name,B", [("celeba64", 32), ("celebaHQ", 8)])
def test_full_width_encoder_vs_fp64(gpu_device, monkeypatch, name, B):
    from damc import amortizer, synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    # the library's weight packing (w_src, extra workgroups of the first layer's launch on CelebA-64's two-pass path)
    # reports any workgroup outside its list; the call then fails instead of returning xemb
    monkeypatch.setenv("DAMC_ENC_PACK_CHECK", "1")

    hw = GEN[name][3]
    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 0, (B, 3, hw, hw))).to(gpu_device)
    got = amortizer.encoder_forward(enc, x).cpu().numpy()
    with torch.no_grad():
        e32 = orc.encoder_forward(enc.cpu(), x.cpu()).numpy()
        e64 = orc.encoder_forward(enc.double(), x.cpu().double()).numpy()
    _check("Encoder_%s nif=64 B=%d xemb" % (name, B), got, e32, e64, 1e-7)


def test_encoder_limb_engine_vs_fp32_engine_b128(gpu_device):
    """The bench's Encoder_cifar10(nif=64) at B=128: the default engine (the k4 s2 and the final convs on the limb
    engine) and the fp32-MFMA engine (damc._lib.exact_fp32) against fp64, both within 3x the fp32 reference's."""
    from damc import _lib, amortizer, synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    B = 128
    enc = synth.load_into(dn.Encoder_cifar10(nc=3, nemb=1024, nif=64), 3).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 1, (B, 3, 32, 32))).to(gpu_device)
    got = amortizer.encoder_forward(enc, x).cpu().numpy()
    with _lib.exact_fp32():
        got32 = amortizer.encoder_forward(enc, x).cpu().numpy()
    with torch.no_grad():
        e32 = orc.encoder_forward(enc.cpu(), x.cpu()).numpy()
        e64 = orc.encoder_forward(enc.double(), x.cpu().double()).numpy()
    _check("Encoder_cifar10 nif=64 B=128 xemb, limb engine", got, e32, e64, 1e-7)
    _check("Encoder_cifar10 nif=64 B=128 xemb, fp32 engine", got32, e32, e64, 1e-7)


@pytest.mark.parametrize("name,B", [("cifar10", 128), ("celeba64", 32), ("cifar10", 16)])
def test_encoder_f32a_convs_are_bitwise(gpu_device, monkeypatch, name, B):
    """The encoder's k4 s2 limb convs staging their input as fp32 (gemm.hip X3_F32A, the one-pass norms writing fp32
    in place) against the limb inputs (DAMC_ENC_F32A=0), and the one-pass norms summing the convs' split-K slabs
    themselves (GemmArgs::ksplit_deferred) against the reduce kernel (DAMC_ENC_IN_SLABS=0): the in-register split is
    the producing epilogue's RNE split and the slab sum the reduce's order, so xemb is bitwise the same."""
    from damc import amortizer, synth
    from src import diffusion_net as dn

    hw = GEN[name][3]
    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 3, (B, 3, hw, hw))).to(gpu_device)
    outs = {}
    for f32a in "10":
        for slabs in "10":  # DAMC_ENC_IN_SLABS: the one-pass norm sums the convs' split-K slabs itself
            monkeypatch.setenv("DAMC_ENC_F32A", f32a)
            monkeypatch.setenv("DAMC_ENC_IN_SLABS", slabs)
            outs[f32a + slabs] = amortizer.encoder_forward(enc, x).cpu()
    for k, v in outs.items():
        assert torch.equal(v, outs["00"]), k


@pytest.mark.parametrize("name,B,hw,nc", [("cifar10", 128, 32, 3), ("cifar10", 200, 32, 3), ("celeba64", 32, 64, 3),
                                         ("mnist", 64, 28, 1)])
def test_encoder_dense_head_vs_fp64(gpu_device, monkeypatch, name, B, hw, nc):
    """The last conv as the dense head (encoder.hip enc_head_x3_kernel: the PyTorch weight read as fp32 and split into
    limbs in the kernel, one workgroup per 128 rows x 64 columns x 512-k sign block, slabs summed in order) and on the
    limb GEMM over the packed weight limbs (DAMC_ENC_HEAD=0): both against fp64 within 3x the fp32 reference's distance;
    B = 200 has a partial 128-row block, mnist a 3 x 3 head (K = 4608).  The head's two launches appear in a profile
    of the call as enc_head_x3_kernel / enc_head_reduce_kernel."""
    from damc import amortizer, synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=nc, nemb=1024, nif=64), 3).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 4, (B, nc, hw, hw))).to(gpu_device)
    monkeypatch.setenv("DAMC_ENC_PACK_CHECK", "1")
    outs = {}
    for h in "10":
        monkeypatch.setenv("DAMC_ENC_HEAD", h)
        outs[h] = amortizer.encoder_forward(enc, x).cpu().numpy()
    monkeypatch.setenv("DAMC_ENC_HEAD", "1")
    for env, v in (("DAMC_ENC_HEAD_PD", "1"), ("DAMC_ENC_HEAD_XCD", "0")):  # schedule and tile order only: bitwise
        monkeypatch.setenv(env, v)
        assert np.array_equal(amortizer.encoder_forward(enc, x).cpu().numpy(), outs["1"]), env
    with torch.no_grad():
        e32 = orc.encoder_forward(enc.cpu(), x.cpu()).numpy()
        e64 = orc.encoder_forward(enc.double(), x.cpu().double()).numpy()
    _check("Encoder_%s B=%d xemb, dense head" % (name, B), outs["1"], e32, e64, 1e-7)
    _check("Encoder_%s B=%d xemb, limb GEMM head" % (name, B), outs["0"], e32, e64, 1e-7)
    assert not np.array_equal(outs["1"], outs["0"])  # (the head ran: its K order differs from the GEMM's)


def test_encoder_descriptor_cache_follows_the_parameters(gpu_device, monkeypatch):
    """EncoderPlan caches its descriptor while the parameters keep their storages.  Values rewritten in place (the
    EMA update's .data.copy_, the fp32-packed first layer included) and a parameter replaced by a new tensor are both
    seen: the next call equals a fresh plan's, under the library packing and DAMC_ENC_WSRC=0."""
    from damc import amortizer, synth
    from src import diffusion_net as dn

    for wsrc in "10":
        monkeypatch.setenv("DAMC_ENC_WSRC", wsrc)
        enc = synth.load_into(dn.Encoder_cifar10(nc=3, nemb=1024, nif=64), 3).to(gpu_device).eval()
        x = torch.from_numpy(synth.uniform_f32(13, 5, (16, 3, 32, 32))).to(gpu_device)
        a = amortizer.encoder_forward(enc, x)
        assert torch.equal(amortizer.encoder_forward(enc, x), a)  # (the cached call)
        with torch.no_grad():
            enc.net[0].weight.mul_(0.5)
            enc.net[4].weight.mul_(0.75)
        b = amortizer.encoder_forward(enc, x)
        assert torch.equal(b, amortizer.EncoderPlan(enc).forward(x)) and not torch.equal(a, b)
        last = enc.net[-1]
        last.weight = torch.nn.Parameter(last.weight.detach() * 0.5)
        c = amortizer.encoder_forward(enc, x)
        assert torch.equal(c, amortizer.EncoderPlan(enc).forward(x)) and not torch.equal(b, c)


@pytest.mark.parametrize("name,B", [("cifar10", 128), ("celeba64", 32)])
def test_encoder_library_packed_weights_are_bitwise(gpu_device, monkeypatch, name, B):
    """damc_enc_layer_t.w_src: the library packs every limb layer's PyTorch weight in one launch (extra workgroups of the
    first layer's launch, or a launch of its own before a two-pass first layer), under the packing's status word.  Bitwise the per-layer damc_pack_conv2d_x3 operands (DAMC_ENC_WSRC=0), and a weight
    rewritten in place through .data between calls (the reference's EMA update, train_gen_recon.py:258-261) is seen
    by the next call."""
    from damc import amortizer, synth
    from src import diffusion_net as dn

    hw = GEN[name][3]
    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 2, (B, 3, hw, hw))).to(gpu_device)
    monkeypatch.setenv("DAMC_ENC_PACK_CHECK", "1")
    # (the last conv on the limb GEMM in both: the dense head reads w_src as fp32, test_encoder_dense_head_vs_fp64)
    monkeypatch.setenv("DAMC_ENC_HEAD", "0")
    monkeypatch.setenv("DAMC_ENC_WSRC", "1")
    a = amortizer.encoder_forward(enc, x).cpu()
    monkeypatch.setenv("DAMC_ENC_WSRC", "0")
    b = amortizer.encoder_forward(enc, x).cpu()
    assert torch.equal(a, b)
    with torch.no_grad():
        for m in enc.modules():
            if isinstance(m, torch.nn.Conv2d):
                m.weight.data.copy_(m.weight.data * 0.75)
    b2 = amortizer.encoder_forward(enc, x).cpu()
    monkeypatch.setenv("DAMC_ENC_WSRC", "1")
    a2 = amortizer.encoder_forward(enc, x).cpu()
    assert torch.equal(a2, b2)
    assert not torch.equal(a2, a)


def test_celebaHQ_q_sweep_vs_fp64(gpu_device):
    """CelebA-HQ Q(x) at its per-rank size (B=8 of 64): Encoder_celebaHQ(nif=64) + the 100-step 'large' reverse sweep
    (nxemb 1024, ntemb 128; train_gen_recon.py:360-380 defaults) with injected noise, vs the fp64 oracle."""
    from damc import amortizer, synth
    from oracle import damc_oracle as orc
    from src import diffusion_net as dn

    B, n = 8, 100
    Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=n,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset="celebaHQ")
    synth.load_into(Q, 20)
    Q.to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(14, 0, (B, 3, 256, 256))).to(gpu_device)
    zt0 = torch.from_numpy(synth.normal_f32(15, 0, (B, 128)))
    eps = torch.from_numpy(np.random.default_rng(16).standard_normal((n - 1, B, 128)).astype(np.float32))
    xemb = amortizer.encoder_forward(Q.encoder, x)
    zt = zt0.to(gpu_device)
    amortizer.reverse_sweep(Q, xemb, zt, noise=eps.to(gpu_device))
    args = (n, -5.1, 9.8, "large")
    Qc = Q.cpu()
    with torch.no_grad():
        z32, _ = orc.reverse_sweep(Qc, orc.encoder_forward(Qc.encoder, x.cpu()), zt0, eps, *args)
        Qd = Qc.double()
        z64, _ = orc.reverse_sweep(Qd, orc.encoder_forward(Qd.encoder, x.cpu().double()), zt0.double(), eps.double(),
                                   *args)
    _check("celebaHQ Q(x) 100-step sweep B=8", zt.cpu().numpy(), z32.numpy(), z64.numpy(), 1e-6)


def test_celebaHQ_b64_posterior_step_equals_its_b8_shards(gpu_device):
    """BASELINE config 5 on one GPU: the whole CelebA-HQ B=64 batch takes a full posterior step (with in-kernel noise)
    in one call, and the result is bitwise the eight per-rank B=8 calls of the same chains (chain_base keys the noise
    by global chain index; the B=8 step itself is checked against fp64 in test_full_width_posterior_vs_fp64, and an
    fp64 oracle at B=64 full width would take the CPU tens of minutes).  The B=64 call runs the unsplit limb GEMMs,
    the B=8 calls the split-K ones, so this also checks that the split reproduces the unsplit sums bit for bit at
    K = 16384."""
    from damc import langevin as lv

    G, E, x, z0 = _case("celebaHQ", 64, gpu_device)
    za = z0.clone()
    lv.posterior_langevin(za, x, G, E, 1, 1.0, 0.1, True, seed=123)
    assert torch.isfinite(za).all() and not torch.equal(za, z0)
    parts = []
    for r in range(8):
        zb = z0[8 * r:8 * r + 8].clone()
        lv.posterior_langevin(zb, x[8 * r:8 * r + 8].contiguous(), G, E, 1, 1.0, 0.1, True, seed=123, chain_base=8 * r)
        parts.append(zb)
    assert torch.equal(za, torch.cat(parts))
