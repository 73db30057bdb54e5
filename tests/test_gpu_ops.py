"""GPU: the per-op hooks SURVEY.md §8(b) names — damc_convT_fwd / damc_convT_dgrad (one k4 s2 p1
ConvTranspose2d layer, diffusion_net.py:20-203), damc_denoise_step / damc_q_reverse_sweep (the reverse step,
diffusion_net.py:585-622), damc_ebm_grad (_netE, :207-223), damc_q_encoder_fwd (Encoder_*, :227-372, covered
through damc.amortizer.encoder_forward in test_gpu_amortizer.py) — against fp64 PyTorch references and
against the whole-path entry points they are cut from.

Tolerances: ConvT rel-L2 <= 1e-6 against fp64 (fp32-accurate limb engine, K <= 4096); the single-step
calls reproduce the sweep to rel 1e-6 (same kernels; the per-sweep time-MLP GEMM runs with M = 1 instead
of M = n); the EBM alias is bitwise.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import Q_NAMES, build_q_case, rel_l2

pytestmark = pytest.mark.gpu


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("ngf,layer", [(32, 1), (32, 2), (128, 2)])
def test_convT_hooks_match_fp64(gpu_device, ngf, layer):
    from damc import _lib, plans, synth
    from damc._lib import ptr
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=ngf, nc=3), 0).to(gpu_device).eval()
    gd = plans.generator_plan(G).refresh(gpu_device)
    Ld = gd.layers[layer]
    conv = G.gen[2 * layer]
    assert isinstance(conv, torch.nn.ConvTranspose2d) and Ld.kind == _lib.LAYER_UP2
    B = 4
    g = torch.Generator().manual_seed(5 + layer)
    h = torch.randn(B, Ld.cin, Ld.hin, Ld.win, generator=g, dtype=torch.float64)
    gout = torch.randn(B, Ld.cout, Ld.hout, Ld.wout, generator=g, dtype=torch.float64)
    w = conv.weight.detach().cpu().double()
    b = conv.bias.detach().cpu().double()
    L = _lib.lib()
    nbytes = int(L.damc_convT_workspace_bytes(ctypes.byref(Ld), B))
    assert nbytes > 0
    ws = torch.empty(nbytes, dtype=torch.uint8, device=gpu_device)
    stream = _lib.stream_ptr(gpu_device)
    # forward: lrelu(conv_transpose2d(h) + b)
    hin = _nhwc(h.float()).to(gpu_device)
    out = torch.empty(B, Ld.hout, Ld.wout, Ld.cout, device=gpu_device)
    _lib.check(L.damc_convT_fwd(ctypes.byref(Ld), ptr(hin), B, ptr(out), ptr(ws), nbytes, stream), "convT_fwd")
    ref = F.leaky_relu(F.conv_transpose2d(h.float().double(), w, b, stride=2, padding=1), 0.2)
    assert rel_l2(out.cpu().numpy(), _nhwc(ref).numpy()) < 1e-6
    # input gradient, masked with lrelu' of the previous layer's (activated) output h
    mask = _nhwc(h.float()).to(gpu_device)
    gin = torch.empty(B, Ld.hin, Ld.win, Ld.cin, device=gpu_device)
    gdev = _nhwc(gout.float()).to(gpu_device)
    _lib.check(L.damc_convT_dgrad(ctypes.byref(Ld), ptr(gdev), B, ptr(mask), _lib.ACT_LRELU, 0.2, ptr(gin), ptr(ws),
                                  nbytes, stream), "convT_dgrad")
    gref = F.conv2d(gout.float().double(), w, stride=2, padding=1)
    gref = gref * torch.where(h.float().double() > 0, 1.0, 0.2)
    assert rel_l2(gin.cpu().numpy(), _nhwc(gref).numpy()) < 1e-6
    # unmasked form
    _lib.check(L.damc_convT_dgrad(ctypes.byref(Ld), ptr(gdev), B, None, 0, 0.0, ptr(gin), ptr(ws), nbytes, stream),
               "convT_dgrad")
    assert rel_l2(gin.cpu().numpy(), _nhwc(F.conv2d(gout.float().double(), w, stride=2, padding=1)).numpy()) < 1e-6


@pytest.mark.parametrize("name", Q_NAMES[:2])
def test_denoise_steps_reproduce_the_sweep(gpu_device, name):
    """n single damc_denoise_step calls (injected noise, step index k) == one damc_q_reverse_sweep."""
    from damc import _lib, amortizer
    from damc._lib import ptr

    c = build_q_case(name, gpu_device)
    Q = c["Q"]
    xemb = amortizer.encoder_forward(Q.encoder, c["x"])
    plan = amortizer.DenoiserPlan(Q.p)
    d = plan.pack(gpu_device)
    n, B = int(Q.n_interval), c["zt0"].shape[0]
    coef_h, temb_d = amortizer.cached_step_tables(n, Q.logsnr_min, Q.logsnr_max, Q.var_type, plan.ntemb, gpu_device)
    L = _lib.lib()
    stream = _lib.stream_ptr(gpu_device)
    noise = c["eps"].contiguous()
    # whole sweep under the SURVEY name
    nb = int(L.damc_sweep_workspace_bytes(ctypes.byref(d), B, n))
    ws = torch.empty(nb, dtype=torch.uint8, device=gpu_device)
    z_sweep = c["zt0"].clone()
    _lib.check(L.damc_q_reverse_sweep(ctypes.byref(d), ptr(xemb), ptr(z_sweep), B, n, ptr(temb_d),
                                      coef_h.numpy().ctypes.data_as(ctypes.c_void_p), 1, ptr(noise), 0, 0, None, 0,
                                      ptr(ws), nb, stream), "q_reverse_sweep")
    # the same, one step per call
    nb1 = int(L.damc_sweep_workspace_bytes(ctypes.byref(d), B, 1))
    ws1 = torch.empty(nb1, dtype=torch.uint8, device=gpu_device)
    z = c["zt0"].clone()
    eps = torch.empty_like(z)
    coef_np = np.ascontiguousarray(coef_h.numpy())
    for k in range(n):
        row = coef_np[k:k + 1]
        nk = noise[k] if k < n - 1 else None
        _lib.check(L.damc_denoise_step(ctypes.byref(d), ptr(xemb), ptr(z), B, ptr(temb_d[k:k + 1].contiguous()),
                                       row.ctypes.data_as(ctypes.c_void_p), 1, ptr(nk), 0, k, 0, ptr(eps), ptr(ws1),
                                       nb1, stream), "denoise_step")
        if k == 0:
            assert rel_l2(eps.cpu().numpy(), c["rec"]["q_post_eps3"][0]) < 1e-5
    torch.cuda.synchronize()
    assert rel_l2(z.cpu().numpy(), z_sweep.cpu().numpy()) < 1e-6


def test_ebm_grad_alias_is_bitwise(gpu_device):
    from damc import _lib, plans, synth
    from damc._lib import ptr
    from src import diffusion_net as dn

    E = synth.load_into(dn._netE(nz=128), 10).to(gpu_device).eval()
    ed = plans.ebm_plan(E).refresh(gpu_device)
    z = torch.from_numpy(synth.normal_f32(3, 0, (64, 128))).to(gpu_device)
    L = _lib.lib()
    stream = _lib.stream_ptr(gpu_device)
    e1, g1 = torch.empty(64, device=gpu_device), torch.empty(64, 128, device=gpu_device)
    e2, g2 = torch.empty_like(e1), torch.empty_like(g1)
    _lib.check(L.damc_ebm_energy_grad(ctypes.byref(ed), ptr(z), 64, ptr(e1), ptr(g1), stream), "ebm_energy_grad")
    _lib.check(L.damc_ebm_grad(ctypes.byref(ed), ptr(z), 64, ptr(e2), ptr(g2), stream), "ebm_grad")
    torch.cuda.synchronize()
    assert torch.equal(e1, e2) and torch.equal(g1, g2)


def test_z_update_hook_vs_oracle(gpu_device):
    """damc_z_update (include/damc.h): z <- z - 0.5 s^2 (g + z) (+ s xi), separately rounded as the reference's
    z.data - 0.5*s*s*z_grad and + s*randn (MCMC.py:36-38,62-64) — bitwise against the same fp32 ops on the CPU,
    with injected noise and with the in-kernel Philox draw (= damc_philox_normal's stream)."""
    from damc import langevin as lv

    g0 = torch.Generator().manual_seed(3)
    z0 = torch.randn(37, 128, generator=g0)
    g = torch.randn(37, 128, generator=g0)
    xi = torch.randn(37, 128, generator=g0)
    s = 0.1
    c1 = np.float32(0.5 * s * s)
    want = (z0 - torch.tensor(c1) * (g + z0)) + torch.tensor(np.float32(s)) * xi
    z = z0.to(gpu_device)
    lv.z_update(z, g.to(gpu_device), s, True, noise=xi.to(gpu_device))
    assert torch.equal(z.cpu(), want)
    z = z0.to(gpu_device)
    lv.z_update(z, g.to(gpu_device), s, False)
    assert torch.equal(z.cpu(), z0 - torch.tensor(c1) * (g + z0))
    # in-kernel Philox: the posterior stream of damc_philox_normal at the same (seed, step, chain)
    z = z0.to(gpu_device)
    lv.z_update(z, g.to(gpu_device), s, True, seed=11, step_index=4, chain_base=100)
    xi_k = lv.philox_normal(1, 37, 128, seed=11, device=gpu_device, step_offset=4, chain_base=100)[0].cpu()
    assert torch.equal(z.cpu(), (z0 - torch.tensor(c1) * (g + z0)) + torch.tensor(np.float32(s)) * xi_k)


@pytest.mark.parametrize("cout,cin,k", [(16, 64, 4), (24, 32, 4), (40, 512, 4), (8, 32, 3), (16, 64, 1), (8, 32, 5),
                                         (8, 128, 4), (16, 256, 3), (8, 64, 5), (8, 512, 3), (8, 96, 4)])
def test_pack_conv2d_x3_matches_limb_split(gpu_device, monkeypatch, cout, cin, k):
    """damc_pack_conv2d_x3 (the encoder's per-call weight operand, Encoder_* convs, diffusion_net.py:227-372):
    PyTorch (cout, cin, k, k) -> K-major [co][(ky, kx, ci)] with the odd sign blocks negated, as three RNE bf16
    limbs h = bf16(v), m = bf16(v - h), l = bf16(v - h - m) per 8-value octet; bit-exact against the same split in
    torch (cin % 128 == 0 or cin == 64 takes the LDS-transposing kernel, other k * k % 4 == 0 the tap-vectorised one,
    the rest the per-octet one)."""
    from damc import _lib
    from damc._lib import ptr

    L = _lib.lib()
    g = torch.Generator().manual_seed(cout * 7 + cin + k)
    w = torch.randn(cout, cin, k, k, generator=g) * torch.exp(torch.randn(cout, cin, k, k, generator=g) * 3)
    for walk in ("0", "1"):  # the opt-in 4 x 4 conv walk (DAMC_ENC_WALK=1, round 6) and the default tap-major order
        monkeypatch.setenv("DAMC_ENC_WALK", walk)
        _check_pack_conv2d_x3(L, w, gpu_device, cout, cin, k)


def _check_pack_conv2d_x3(L, w, gpu_device, cout, cin, k):
    from damc import _lib
    from damc._lib import ptr

    nb = int(L.damc_conv2d_x3_bytes(cout, cin, k))
    assert nb == cout * k * k * cin * 6
    out = torch.zeros(nb // 2, dtype=torch.int16, device=gpu_device)
    wd = w.to(gpu_device)
    _lib.check(L.damc_pack_conv2d_x3(ptr(wd), cout, cin, k, ptr(out), _lib.stream_ptr(gpu_device)), "pack x3")
    torch.cuda.synchronize()
    K = k * k * cin
    v = w.permute(0, 2, 3, 1).reshape(cout, K)
    if L.damc_x3_conv_walk(k, cin):  # 4 x 4 convs: slice-major, parity-grouped taps (damc_x3_conv_walk, round 6)
        walk = []
        for sl in range(cin // 32):
            for pos in range(16):
                c, j = pos // 4, pos % 4
                tap = ((c >> 1) + 2 * (j >> 1)) * 4 + (c & 1) + 2 * (j & 1)
                walk += [tap * cin + 32 * sl + i for i in range(32)]
        v = v[:, torch.tensor(walk)]
    nk = int(L.damc_x3_sign_block())  # k per sign block
    sg = torch.where((torch.arange(K) // nk) % 2 == 1, -1.0, 1.0)
    v = v * sg
    h = v.to(torch.bfloat16)
    r1 = v - h.float()
    m = r1.to(torch.bfloat16)
    lo = (r1 - m.float()).to(torch.bfloat16)
    want = torch.stack([t.view(torch.int16).reshape(cout, K // 8, 8) for t in (h, m, lo)], dim=2).reshape(-1)
    assert torch.equal(out.cpu(), want)


@pytest.mark.parametrize("cls,ngf", [("_netG_cifar10", 128), ("_netG_celebaHQ", 64), ("_netG_mnist", 64)])
def test_tiled_weight_packing_is_bitwise_the_elementwise_packing(gpu_device, monkeypatch, cls, ngf):
    """damc_pack_generator_layer's LDS-tiled path (fp32 + x3 limbs in one pass) writes exactly the bytes of the
    element-wise packing + launch_split_x3_conv (DAMC_PACK_TILED=0) for every layer of the generators."""
    from damc import plans, synth
    from src import diffusion_net as dn

    G = synth.load_into(getattr(dn, cls)(nz=128, ngf=ngf, nc=3), 3).to(gpu_device).eval()
    plan = plans.generator_plan(G)
    got = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DAMC_PACK_TILED", mode)
        plan.refresh(gpu_device)
        torch.cuda.synchronize()
        got[mode] = [(wf.clone(), None if wb is None else wb.clone()) for wf, wb in plan.buffers]
    for i, ((f0, b0), (f1, b1)) in enumerate(zip(got["0"], got["1"])):
        assert torch.equal(f0, f1), f"layer {i} forward packing"
        assert (b0 is None) == (b1 is None)
        if b0 is not None:
            assert torch.equal(b0, b1), f"layer {i} backward packing"
