"""GPU: the G update of a training iteration (workspace/train_gen_recon.py:222-231) on the HIP path.

``_netG_*.forward`` on ROCm tensors runs damc.training (forward kernels + the HIP training backward:
limb-engine weight gradients of the k4 s2 p1 / first layers, the direct output-layer weight gradient,
bias column sums).  Checked against (a) the reference's own autograd gradients (golden subsamples and
full norms, tests/golden/*_gtrain.npz) and (b) the oracle's explicit backward on the same inputs.

Tolerance: rel-L2 <= 2e-5 per parameter tensor against the reference (fp32 results summed in a different
order over up to B*H*W = 131K terms; the limb engine's products carry fp32's 24 significand bits,
gemm.hip); at full width, accuracy-relative against fp64 (see the full-width test).
"""
import numpy as np
import pytest
import torch

from conftest import G_NAMES, gtrain_check, gtrain_inputs, rel_l2
from oracle import damc_oracle as orc

pytestmark = pytest.mark.gpu
TOL = 2e-5


def _hip_grads(G, z, x, want_z=False):
    G.train()
    for p in G.parameters():
        p.grad = None
    zz = z.clone().requires_grad_(want_z)
    x_hat = G(zz)
    loss = torch.sum((x_hat - x) ** 2, dim=[1, 2, 3]).mean()
    loss.backward()
    torch.cuda.synchronize()
    return [p.grad.detach().cpu().numpy() for p in G.parameters()], float(loss.detach()), (zz.grad if want_z else None)


@pytest.mark.parametrize("name", G_NAMES)
def test_generator_train_grads_match_reference(gpu_device, name):
    G, z0, x, rec, meta = gtrain_inputs(name)
    G = G.to(gpu_device)
    grads, loss, _ = _hip_grads(G, z0.to(gpu_device), x.to(gpu_device))
    assert abs(loss - float(rec["g_loss"])) / float(rec["g_loss"]) < 1e-6
    worst = gtrain_check(grads, rec, meta, TOL)
    print("%s worst rel err vs reference %.2e" % (name, worst))


@pytest.mark.parametrize("B", [40, 128])
def test_generator_train_grads_full_width_vs_oracle(gpu_device, B):
    """CIFAR-10 _netG_cifar10(ngf=128) at a ragged batch (B=40 -> padded to 64) and at the bench batch.

    As in test_cifar_b128_step_vs_oracle, the full-width random-weight generator is ill-conditioned
    (pre-activations within rounding of zero flip LReLU' between any two fp32 evaluations): the fp32
    restatement of the reference's arithmetic itself sits up to ~1e-3 from fp64 on the first layers.
    The criterion is accuracy-relative: per tensor, the HIP gradient's distance to an fp64 evaluation
    stays within 3x the fp32 reference arithmetic's distance to it (+ a 1e-6 floor)."""
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0)
    z0 = torch.from_numpy(synth.normal_f32(2, 7, (B, 128)))
    x = torch.from_numpy(synth.uniform_f32(1, 7, (B, 3, 32, 32)))
    refs = []
    for dt in (torch.float32, torch.float64):
        L = orc.generator_layers(G, dt)
        zz, xx = z0.to(dt), x.to(dt)
        xh = orc.generator_sample(L, zz)
        g, gz_ref, _ = orc.generator_train_grads(L, zz, 2.0 * (xh - xx) / B)
        refs.append(([t for gw, gb in g for t in (gw, gb)] + [gz_ref]))
    Gd = G.to(gpu_device)
    grads, _, gz = _hip_grads(Gd, z0.to(gpu_device), x.to(gpu_device), want_z=True)
    for k, (hip, r32, r64) in enumerate(zip(grads + [gz.cpu().numpy()], *refs)):
        e_hip, e32 = rel_l2(hip, r64.numpy()), rel_l2(r32.numpy(), r64.numpy())
        print("B=%d tensor %d: |hip - fp64| %.2e, |fp32 ref - fp64| %.2e" % (B, k, e_hip, e32))
        assert e_hip <= 3 * e32 + 1e-6, (k, e_hip, e32)


def test_generator_train_backward_is_deterministic(gpu_device):
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_svhn(nz=100, ngf=32, nc=3), 0).to(gpu_device)
    z = torch.from_numpy(synth.normal_f32(2, 9, (48, 100))).to(gpu_device)
    x = torch.from_numpy(synth.uniform_f32(1, 9, (48, 3, 32, 32))).to(gpu_device)
    a, _, _ = _hip_grads(G, z, x)
    b, _, _ = _hip_grads(G, z, x)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_generator_forward_no_grad_is_hip(gpu_device):
    """Under no_grad the drop-in forward is the plain HIP forward (gen_samples path) and matches the oracle."""
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(dn._netG_celeba64(nz=100, ngf=16, nc=3), 0)
    z = torch.from_numpy(synth.normal_f32(2, 11, (5, 100)))
    ref = orc.generator_sample(orc.generator_layers(G), z)
    with torch.no_grad():
        out = G.to(gpu_device)(z.to(gpu_device).reshape(5, 100, 1, 1))
    assert not out.requires_grad
    assert rel_l2(out.cpu().numpy(), ref.numpy()) < 1e-5


# ------------------------------------------------------------------------------------------ Q update
@pytest.mark.parametrize("name", ["q_cifar10_s", "q_svhn_s", "q_mnist_s", "q_cifar10_full"])
def test_q_update_matches_reference(gpu_device, name):
    """The Q update's loss and gradients (train_gen_recon.py:211-217) with the denoiser forward/backward on
    libdamc (damc_denoiser_train_*), the encoder / prior_emb / noising on PyTorch, vs the reference's autograd
    on the same injected noise and a mixed mask.  Tolerance as for the G update."""
    from conftest import qtrain_run

    from damc import training

    calls = []
    orig = training.encoder_apply
    training.encoder_apply = lambda enc, x: calls.append(1) or orig(enc, x)
    try:
        loss, grads, rec, meta = qtrain_run(name, gpu_device)
    finally:
        training.encoder_apply = orig
    # the encoder ran on libdamc for every topology whose convs the C side covers (mnist's 7 -> 3 stride-2
    # conv is not a k4 s2 p1 with H = 2 Ho: stock PyTorch there)
    assert bool(calls) == (name != "q_mnist_s")
    assert rel_l2(loss, rec["loss"]) < 1e-5
    # 1e-4: the time embedding sin/cos(1000 * f * t) (SinusoidalPosEmb, arguments up to ~1000 rad, whose own
    # fp32 rounding is ~3e-5 absolute) is torch's on each device, GPU vs the reference's CPU; with B = 3-4
    # samples that difference reaches time_mlp[1].weight's gradient unaveraged (its norm agrees to ~1e-6)
    worst = gtrain_check(grads, rec, meta, 1e-4)
    print("%s worst rel err vs reference %.2e" % (name, worst))


def test_denoiser_train_vs_autograd_b128(gpu_device):
    """Bench-size Q update (B=128, nz=128, nxemb=1024, ntemb=128, nf=4): HIP denoiser forward/backward vs
    PyTorch autograd of the same module on the same device, all outputs and every parameter gradient."""
    from damc import synth, training
    from src import diffusion_net as dn

    B = 128
    p = synth.load_into(dn.Diffusion_UnetA(nz=128, nxemb=1024, ntemb=128, residual=True, nf=4), 3).to(gpu_device)
    zt = torch.from_numpy(synth.normal_f32(5, 0, (B, 128))).to(gpu_device)
    logsnr = torch.from_numpy(synth.uniform_f32(5, 1, (B,), -5.0, 9.0)).to(gpu_device)
    xe = torch.from_numpy(synth.normal_f32(5, 2, (B, 1024))).to(gpu_device)
    w = torch.from_numpy(synth.normal_f32(5, 3, (B, 128))).to(gpu_device)

    def run(hip):
        p.zero_grad()
        x = xe.clone().requires_grad_(True)
        if hip:
            out = p(zt, logsnr.clone(), x)
        else:
            t_in = torch.arctan(torch.exp(-0.5 * torch.clamp(logsnr, -20.0, 20.0))) / (0.5 * np.pi)
            out = _stock_denoiser(p, zt, t_in, x)
        (out * w).sum().backward()
        return out.detach(), x.grad.detach(), [q.grad.detach().clone() for q in p.parameters()]

    o1, gx1, g1 = run(True)
    o0, gx0, g0 = run(False)
    assert rel_l2(o1.cpu().numpy(), o0.cpu().numpy()) < 1e-5
    assert rel_l2(gx1.cpu().numpy(), gx0.cpu().numpy()) < 2e-5
    for k, (a, b) in enumerate(zip(g1, g0)):
        assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) < 2e-5, k
    assert training._DenoiserTrainFn is not None


def _stock_denoiser(p, z, t_in, xemb):
    """Diffusion_UnetA.forward's stock-PyTorch body (the drop-in's non-ROCm branch), for autograd."""
    import torch.nn.functional as F

    temb = p.time_mlp(t_in)
    ctx = torch.cat([temb, xemb], dim=1)
    skips, out = [], p.input_emb(z)
    for layer in p.in_layers:
        out = layer(ctx=ctx, x=out)
        skips.append(out)
        out = F.leaky_relu(out, negative_slope=0.01)
    out = p.mid_layers[0](ctx=ctx, x=out)
    for layer in p.out_layers:
        out = layer(ctx=ctx, x=F.leaky_relu(torch.cat([out, skips.pop()], dim=1), negative_slope=0.01))
    return z + out if p.residual else out


def test_encoder_train_vs_autograd_b128(gpu_device):
    """Bench-size encoder training (CIFAR-10 Encoder, nif 64, nemb 1024, B=128): libdamc forward/backward
    (InstanceNorm backward, k4 s2 p1 convs through the limb engine with swapped roles, first and last conv)
    against an fp64 evaluation of the same module, accuracy-relative: per tensor, the HIP result's distance to
    fp64 stays within 3x the distance of PyTorch's own fp32 autograd (MIOpen) to fp64 (the four InstanceNorm
    backwards subtract per-channel means, so the first layers' gradients carry cancellation in any fp32
    evaluation).  Floor: 1e-3 x the largest gradient norm (conv biases feeding InstanceNorm have an
    analytically zero gradient)."""
    import copy

    from damc import synth, training
    from src import diffusion_net as dn

    enc = synth.load_into(dn.Encoder_cifar10(nc=3, nemb=1024, nif=64), 4).to(gpu_device).train()
    enc64 = copy.deepcopy(enc).double()
    x = torch.from_numpy(synth.uniform_f32(6, 0, (128, 3, 32, 32))).to(gpu_device)
    w = torch.from_numpy(synth.normal_f32(6, 1, (128, 1024))).to(gpu_device)
    assert training.encoder_train_supported(enc, x)

    def run(net, hip, xx, ww):
        net.zero_grad()
        if hip:
            out = net(xx)
        else:
            with training.stock_pytorch():
                out = net(xx)
        (out * ww).sum().backward()
        return out.detach().double(), [p.grad.detach().double().clone() for p in net.parameters()]

    o1, g1 = run(enc, True, x, w)
    o0, g0 = run(enc, False, x, w)
    o64, g64 = run(enc64, False, x.double(), w.double())
    assert float((o1 - o64).norm() / o64.norm()) <= 3 * float((o0 - o64).norm() / o64.norm()) + 1e-6
    floor = 1e-3 * max(float(b.norm()) for b in g64)
    for k, (a, b, r) in enumerate(zip(g1, g0, g64)):
        den = max(float(r.norm()), floor)
        e_hip, e32 = float((a - r).norm()) / den, float((b - r).norm()) / den
        print("encoder tensor %d: |hip - fp64| %.2e, |torch fp32 - fp64| %.2e" % (k, e_hip, e32))
        assert e_hip <= 3 * e32 + 1e-6, (k, e_hip, e32)
