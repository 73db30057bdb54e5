"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

CPU restatement (PyTorch-CPU, fp32 by default, fp64 on request) of the reference's
diffusion-amortized Langevin inner loop.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker /
the timed CPU baseline.  The product (damc + libdamc.so) never calls it.

Pinned against golden vectors captured from the reference itself
(tests/golden/make_golden.py -> tests/golden/*.npz; checked by
tests/test_oracle_golden.py).  Gradients are written out explicitly (no
autograd), so the restatement is an independent derivation of the reference's
autograd result:

  posterior U(z) = |G(z)-x|^2/(2 s^2) + sum E(z) + |z|^2/2      workspace/src/MCMC.py:55-60
  prior     U(z) = sum E(z) + |z|^2/2                             workspace/src/MCMC.py:32-34
  update    z <- z - 0.5*s*s*grad (+ s*xi)                        workspace/src/MCMC.py:36-38,62-64

Generator dgrad identity: conv_transpose2d is the adjoint of conv2d with the same
weight/stride/padding, so d<dy, convT(h)>/dh = conv2d(dy, W, stride, padding).
"""
import math

import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# network descriptions (plain dicts of tensors; built from any nn.Module with the
# reference's structure, i.e. reference classes or the damc drop-in classes)
# --------------------------------------------------------------------------------------


def _act_of(mod):
    if isinstance(mod, torch.nn.LeakyReLU):
        return ("lrelu", float(mod.negative_slope))
    if isinstance(mod, torch.nn.ReLU):
        return ("lrelu", 0.0)
    if isinstance(mod, torch.nn.Tanh):
        return ("tanh", 0.0)
    return None


def generator_layers(G, dtype=torch.float32):
    """Ordered layer list of a generator: reference `_netG_*.gen` (diffusion_net.py:20-203)
    or the toy MLP `G.net` (toy_example.py:22-47)."""
    seq = G.gen if hasattr(G, "gen") else G.net
    layers = []
    for m in seq:
        if isinstance(m, torch.nn.ConvTranspose2d):
            layers.append(dict(kind="convT", W=m.weight.detach().cpu().to(dtype),
                               b=None if m.bias is None else m.bias.detach().cpu().to(dtype),
                               stride=m.stride[0], pad=m.padding[0], act=("none", 0.0)))
        elif isinstance(m, torch.nn.Linear):
            layers.append(dict(kind="linear", W=m.weight.detach().cpu().to(dtype),
                               b=None if m.bias is None else m.bias.detach().cpu().to(dtype),
                               act=("none", 0.0)))
        else:
            a = _act_of(m)
            assert a is not None and layers, m
            layers[-1]["act"] = a
    return layers


def ebm_params(E, dtype=torch.float32):
    """`_netE.ebm` = Linear, LReLU(.2), Linear, LReLU(.2), Linear (diffusion_net.py:207-223)."""
    lin = [m for m in E.ebm if isinstance(m, torch.nn.Linear)]
    return [(m.weight.detach().cpu().to(dtype), m.bias.detach().cpu().to(dtype)) for m in lin]


def _apply_act(a, act):
    kind, slope = act
    if kind == "lrelu":
        return F.leaky_relu(a, slope)
    if kind == "tanh":
        return torch.tanh(a)
    return a


def _act_backward(d, h, act):
    """d * act'(.) expressed through the post-activation h (single fused ATen pass, as autograd)."""
    kind, slope = act
    if kind == "lrelu":
        return torch.ops.aten.leaky_relu_backward(d, h, slope, True)
    if kind == "tanh":
        return torch.ops.aten.tanh_backward(d, h)
    return d


def _act_grad_from_out(h, act):
    kind, slope = act
    if kind == "lrelu":
        return torch.where(h > 0, torch.ones_like(h), torch.full_like(h, slope))
    if kind == "tanh":
        return 1.0 - h * h
    return torch.ones_like(h)


def generator_forward(layers, z):
    """Returns the list of post-activation outputs; [-1] is x_hat (diffusion_net.py:49-51)."""
    h = z
    hs = []
    for i, L in enumerate(layers):
        if L["kind"] == "convT":
            if i == 0:
                h = h.reshape(len(h), -1, 1, 1)
            a = F.conv_transpose2d(h, L["W"], L["b"], stride=L["stride"], padding=L["pad"])
        else:
            a = F.linear(h, L["W"], L["b"])
        h = _apply_act(a, L["act"])
        hs.append(h)
    return hs


def generator_vjp(layers, hs, delta_last):
    """J_G(z)^T applied to dL/da_last (the pre-activation gradient of the last layer)."""
    d = delta_last
    for i in range(len(layers) - 1, -1, -1):
        L = layers[i]
        if L["kind"] == "convT":
            # input gradient of the transposed conv (= conv2d(d, W, stride, pad)), through ATen's
            # convolution_backward — the kernel the reference's autograd dispatches to, so the CPU
            # baseline times the same arithmetic the reference runs (no autograd graph involved)
            inp = hs[i - 1] if i > 0 else None
            if inp is None:
                inp = torch.empty(d.shape[0], L["W"].shape[0], 1, 1, dtype=d.dtype)
            dh = torch.ops.aten.convolution_backward(
                d, inp, L["W"], None, [L["stride"]] * 2, [L["pad"]] * 2, [1, 1], True, [0, 0], 1,
                [True, False, False])[0]
        else:
            dh = d @ L["W"]
        if i == 0:
            return dh.reshape(len(dh), -1)
        d = _act_backward(dh, hs[i - 1], layers[i - 1]["act"])
    raise AssertionError


def generator_train_grads(layers, z, grad_xhat):
    """The G update's gradients (workspace/train_gen_recon.py:222-231: x_hat = G(z), loss.backward()):
    given dL/dx_hat, per layer (dL/dW, dL/db) and dL/dz.  Explicit backward through ATen's
    convolution_backward (the kernel the reference's autograd dispatches to for ConvTranspose2d,
    diffusion_net.py:20-203) and the Linear identities (toy G, toy_example.py:22-47)."""
    hs = generator_forward(layers, z)
    d = _act_backward(grad_xhat, hs[-1], layers[-1]["act"])
    grads = [None] * len(layers)
    gz = None
    for i in range(len(layers) - 1, -1, -1):
        L = layers[i]
        if L["kind"] == "convT":
            inp = hs[i - 1] if i > 0 else z.reshape(len(z), -1, 1, 1)
            gi, gw, gb = torch.ops.aten.convolution_backward(
                d, inp, L["W"], [L["W"].shape[1]], [L["stride"]] * 2, [L["pad"]] * 2, [1, 1], True, [0, 0], 1,
                [True, True, L["b"] is not None])
        else:
            inp = hs[i - 1] if i > 0 else z
            gw = d.t() @ inp
            gb = d.sum(0) if L["b"] is not None else None
            gi = d @ L["W"]
        grads[i] = (gw, gb)
        if i > 0:
            d = _act_backward(gi, hs[i - 1], layers[i - 1]["act"])
        else:
            gz = gi.reshape(len(z), -1)
    return grads, gz, hs[-1]


def likelihood_grad(layers, z, x, sigma):
    """grad_z |G(z)-x|^2/(2 sigma^2) and the energy value (MCMC.py:55-56)."""
    hs = generator_forward(layers, z)
    xh = hs[-1]
    r = xh - x
    delta = (r / (sigma * sigma)) * _act_grad_from_out(xh, layers[-1]["act"])
    lik = (r * r).sum() / (2.0 * sigma * sigma)
    return generator_vjp(layers, hs, delta), lik, xh


def ebm_energy_grad(params, z, slope=0.2):
    """E(z) per row and grad_z sum E (diffusion_net.py:212-223)."""
    (W1, b1), (W2, b2), (W3, b3) = params
    a1 = F.linear(z, W1, b1)
    h1 = torch.where(a1 > 0, a1, slope * a1)
    a2 = F.linear(h1, W2, b2)
    h2 = torch.where(a2 > 0, a2, slope * a2)
    e = F.linear(h2, W3, b3).reshape(-1)
    m2 = torch.where(a2 > 0, 1.0, slope).to(z.dtype)
    m1 = torch.where(a1 > 0, 1.0, slope).to(z.dtype)
    g2 = m2 * W3.reshape(1, -1)
    g1 = (g2 @ W2) * m1
    return e, g1 @ W1


def posterior_langevin(layers, ebm, z0, x, n_steps, sigma, step, noise=None, ebm_on=True):
    """sample_langevin_post_z_with_prior (MCMC.py:48-74); noise: (n_steps, B, nz) or None."""
    z = z0.clone()
    c = 0.5 * step * step
    for i in range(n_steps):
        gl, _, _ = likelihood_grad(layers, z, x, sigma)
        g = gl + z
        if ebm_on:
            g = g + ebm_energy_grad(ebm, z)[1]
        z = z - c * g
        if noise is not None:
            z = z + step * noise[i]
    return z


def prior_langevin(ebm, z0, n_steps, step, noise=None):
    """sample_langevin_prior_z (MCMC.py:27-46)."""
    z = z0.clone()
    c = 0.5 * step * step
    for i in range(n_steps):
        g = ebm_energy_grad(ebm, z)[1] + z
        z = z - c * g
        if noise is not None:
            z = z + step * noise[i]
    return z


def generator_sample(layers, z):
    return generator_forward(layers, z)[-1]


# --------------------------------------------------------------------------------------
# amortizer Q: encoder + latent-diffusion reverse sweep (diffusion_net.py:227-622)
# --------------------------------------------------------------------------------------


def encoder_forward(enc, x):
    """Encoder_*: [Conv2d -> InstanceNorm2d(affine, eps 1e-5) -> LReLU(.2)]* -> Conv2d."""
    h = x
    mods = list(enc.net)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, torch.nn.Conv2d):
            h = F.conv2d(h, m.weight.detach().to(h.dtype), m.bias.detach().to(h.dtype),
                         stride=m.stride, padding=m.padding)
        elif isinstance(m, torch.nn.InstanceNorm2d):
            mu = h.mean(dim=(2, 3), keepdim=True)
            var = ((h - mu) ** 2).mean(dim=(2, 3), keepdim=True)
            h = (h - mu) / torch.sqrt(var + m.eps)
            h = h * m.weight.detach().to(h.dtype).view(1, -1, 1, 1) + m.bias.detach().to(h.dtype).view(1, -1, 1, 1)
        elif isinstance(m, torch.nn.LeakyReLU):
            h = torch.where(h > 0, h, h * m.negative_slope)
        i += 1
    return h.reshape(len(x), -1)


def logsnr_schedule(t, logsnr_min, logsnr_max):
    """diffusion_helper_func.py:41-50 (evaluated in t's dtype, op for op, as the reference does)."""
    lmin = logsnr_min * torch.ones_like(t)
    lmax = logsnr_max * torch.ones_like(t)
    b = torch.atan(torch.exp(-0.5 * lmax))
    a = torch.atan(torch.exp(-0.5 * lmin)) - b
    return -2.0 * torch.log(torch.tan(a * t + b))


def _lin(m, x):
    return F.linear(x, m.weight.detach().to(x.dtype), None if m.bias is None else m.bias.detach().to(x.dtype))


def _silu(x):
    return x * torch.sigmoid(x)


def concat_squash(blk, ctx, x):
    """ConcatSquashLinearSkipCtx.forward (diffusion_net.py:439-445)."""
    c = _silu(_lin(blk._layer_ctx[1], _silu(ctx)))
    gate = torch.sigmoid(_lin(blk._hyper_gate, c))
    bias = _lin(blk._hyper_bias, c)
    return _lin(blk._layer[0], x) * gate + bias + _lin(blk._skip, x)


def denoiser_forward(p, z, logsnr, xemb):
    """Diffusion_UnetA.forward (diffusion_net.py:501-533)."""
    li = torch.atan(torch.exp(-0.5 * torch.clamp(logsnr, -20.0, 20.0))) / (0.5 * math.pi)
    half = p.ntemb // 2
    freqs = torch.exp(torch.arange(half, dtype=z.dtype) * -(math.log(10000) / (half - 1)))
    e = (li * 1000.0)[:, None] * freqs[None, :]
    temb = torch.cat([e.sin(), e.cos()], dim=-1)
    temb = _lin(p.time_mlp[3], _silu(_lin(p.time_mlp[1], temb)))
    ctx = torch.cat([temb, xemb], dim=1)
    zb = z @ p.B.detach().to(z.dtype)
    out = torch.cat([torch.sin(2 * math.pi * zb), torch.cos(2 * math.pi * zb), z], dim=1)
    lrelu = lambda v: torch.where(v > 0, v, 0.01 * v)  # noqa: E731
    hs = []
    for blk in p.in_layers:
        out = concat_squash(blk, ctx, out)
        hs.append(out)
        out = lrelu(out)
    out = concat_squash(p.mid_layers[0], ctx, out)
    for blk in p.out_layers:
        out = lrelu(torch.cat([out, hs.pop()], dim=1))
        out = concat_squash(blk, ctx, out)
    return z + out if p.residual else out


def reverse_sweep(Q, xemb, zt, eps_noise, n_interval, logsnr_min, logsnr_max, var_type, with_noise=True):
    """_netQ_U.forward loop (diffusion_net.py:595-622); eps_noise: (n_interval-1, B, nz)."""
    b = len(zt)
    eps_log = []
    k = 0
    for i in reversed(range(n_interval)):
        it = torch.full((b,), float(i), dtype=torch.float32)
        lt = logsnr_schedule(it / (n_interval - 1.0), logsnr_min, logsnr_max).to(zt.dtype)
        ls = logsnr_schedule(torch.clamp(it - 1.0, min=0.0) / (n_interval - 1.0), logsnr_min, logsnr_max).to(zt.dtype)
        eps = denoiser_forward(Q.p, zt, lt, xemb)
        eps_log.append(eps)
        lt, ls = lt[:, None], ls[:, None]
        pred = torch.sqrt(1.0 + torch.exp(-lt)) * (zt - eps * torch.rsqrt(1.0 + torch.exp(lt)))
        if i == 0:
            zt = pred
        else:
            alpha_st = torch.sqrt((1.0 + torch.exp(-lt)) / (1.0 + torch.exp(-ls)))
            alpha_s = torch.sqrt(torch.sigmoid(ls))
            r = torch.exp(lt - ls)
            omr = -torch.expm1(lt - ls)
            mean = r * alpha_st * zt + omr * alpha_s * pred
            if var_type == "large":
                var = omr * torch.sigmoid(-lt)
            else:
                a_t, a_s = torch.sigmoid(lt), torch.sigmoid(ls)
                var = (1.0 - a_s) / (1.0 - a_t) * (1 - a_t / a_s)
            zt = mean + torch.sqrt(var) * eps_noise[k] if with_noise else mean
            k += 1
    return zt, eps_log


def prior_embedding(Q, noise):
    """prior_emb: Linear(nz,128) -> LeakyReLU(0.01) -> Linear(128,nxemb) (diffusion_net.py:577-581)."""
    h = _lin(Q.prior_emb[0], noise)
    h = torch.where(h > 0, h, 0.01 * h)
    return _lin(Q.prior_emb[2], h)
