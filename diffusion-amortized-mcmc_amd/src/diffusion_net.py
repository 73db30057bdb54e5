"""Drop-in for workspace/src/diffusion_net.py (the reference's network module).

Same class names, constructor signatures and ``state_dict`` keys/order as the reference, so
reference checkpoints load unchanged (workspace/train_gen_recon.py:284-294).  The nets are
built from compact spec tables.  The hot path — Langevin sampling and the amortizer's
reverse sweep — runs on the HIP kernels: ``_netQ_U.forward`` dispatches to
``damc.amortizer`` and ``src.MCMC`` to ``damc.langevin``.  ``_netG_*.forward`` on ROCm
tensors runs on libdamc too, with a HIP backward for the G update (``damc.training``).
``forward`` of E / encoders / denoiser stays stock PyTorch (their training updates are
outside the hot path).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .diffusion_helper_func import diffusion_forward, logsnr_schedule_fn  # noqa: F401
from .diffusion_helper_func import *  # noqa: F401,F403  (reference re-exports the helpers)


def spectral_norm(module, mode=True):
    return nn.utils.spectral_norm(module) if mode else module


# ------------------------------------------------------------------------------ generators
# (first kernel, hidden channel multipliers of ngf, (last kernel, stride, pad))
_G_TOPOLOGY = {
    "cifar10": (8, (8, 4, 2), (3, 1, 1)),   # diffusion_net.py:20-51
    "svhn": (4, (8, 4, 2), (4, 2, 1)),      # :53-84
    "celeba64": (4, (8, 4, 2, 1), (4, 2, 1)),  # :86-122
    "celebaHQ": (4, (16, 8, 4, 4, 2, 1), (4, 2, 1)),  # :124-170
    "mnist": (7, (8, 4, 2), (3, 1, 1)),     # :172-203
}


def _deconv_stack(nz, ngf, nc, topo, use_spc_norm):
    k0, mults, (kl, sl, pl) = topo
    chans = [ngf * m for m in mults]
    act = nn.LeakyReLU(0.2)
    mods = [spectral_norm(nn.ConvTranspose2d(nz, chans[0], k0, 1, 0, bias=True), use_spc_norm), act]
    for cin, cout in zip(chans[:-1], chans[1:]):
        mods += [spectral_norm(nn.ConvTranspose2d(cin, cout, 4, 2, 1, bias=True), use_spc_norm), act]
    mods += [spectral_norm(nn.ConvTranspose2d(chans[-1], nc, kl, sl, pl), use_spc_norm), nn.Tanh()]
    return nn.Sequential(*mods)


class _GeneratorBase(nn.Module):
    TOPOLOGY = None

    def __init__(self, nz, ngf, nc, use_spc_norm=False):
        super().__init__()
        self.nz = nz
        self._spc = bool(use_spc_norm)
        self.gen = _deconv_stack(nz, ngf, nc, _G_TOPOLOGY[self.TOPOLOGY], use_spc_norm)

    def forward(self, z):
        # ROCm tensors run on libdamc: the forward, and under autograd the training backward
        # (damc.training: dL/dW, dL/db, dL/dz for the G update, train_gen_recon.py:222-231).
        # Spectral-norm generators (use_spc_norm=True, default False) run their forward on the stock layers (the
        # Langevin chains, gen_samples and the sweeps take them on libdamc in eval mode: damc.plans._live_weight).
        if z.is_cuda and not self._spc:
            from damc import training

            if training.ENABLED:
                return training.generator_apply(self, z)
        return self.gen(z.reshape(z.shape[0], self.nz, 1, 1))


class _netG_cifar10(_GeneratorBase):
    TOPOLOGY = "cifar10"

    def __init__(self, nz=128, ngf=128, nc=3, use_spc_norm=False):
        super().__init__(nz, ngf, nc, use_spc_norm)


class _netG_svhn(_GeneratorBase):
    TOPOLOGY = "svhn"

    def __init__(self, nz=100, ngf=64, nc=3, use_spc_norm=False):
        super().__init__(nz, ngf, nc, use_spc_norm)


class _netG_celeba64(_GeneratorBase):
    TOPOLOGY = "celeba64"

    def __init__(self, nz=100, ngf=128, nc=3, use_spc_norm=False):
        super().__init__(nz, ngf, nc, use_spc_norm)


class _netG_celebaHQ(_GeneratorBase):
    TOPOLOGY = "celebaHQ"

    def __init__(self, nz=128, ngf=128, nc=3, use_spc_norm=False):
        super().__init__(nz, ngf, nc, use_spc_norm)


class _netG_mnist(_GeneratorBase):
    TOPOLOGY = "mnist"

    def __init__(self, nz=100, ngf=128, nc=1, use_spc_norm=False):
        super().__init__(nz, ngf, nc, use_spc_norm)


# --------------------------------------------------------------------------------- latent EBM
class _netE(nn.Module):
    """E(z) = MLP nz -> ndf -> ndf -> nez with LeakyReLU(0.2) (diffusion_net.py:207-223)."""

    def __init__(self, nz=128, ndf=200, nez=1, e_sn=False):
        super().__init__()
        wrap = nn.utils.spectral_norm if e_sn else (lambda m: m)
        act = nn.LeakyReLU(0.2)
        self.ebm = nn.Sequential(wrap(nn.Linear(nz, ndf)), act, wrap(nn.Linear(ndf, ndf)), act,
                                 wrap(nn.Linear(ndf, nez)))

    def forward(self, z):
        if z.is_cuda and torch.is_grad_enabled():
            # ROCm with autograd on (the E update, train_gen_recon.py:233-241): forward and backward on libdamc
            # (damc.training.ebm_apply); None where the C side does not take the module, then the stock layers
            from damc import training

            if training.ENABLED and (z.requires_grad or any(p.requires_grad for p in self.parameters())):
                e = training.ebm_apply(self, z)
                if e is not None:
                    return e
        return self.ebm(z).squeeze()


# ---------------------------------------------------------------------------------- encoders
# (hidden channel multipliers of nif; final conv kernel) — first conv is 3x3 s1 p1, then 4x4 s2 p1
_ENC_TOPOLOGY = {
    "cifar10": ((1, 2, 4, 8), 4),              # diffusion_net.py:227-266
    "celeba64": ((1, 2, 4, 8, 8), 4),          # :268-313
    "celebaHQ": ((1, 2, 4, 4, 8, 8, 8), 4),    # :315-372
    "mnist": ((1, 2, 4, 8), 3),                # :374-413
}


class _EncoderBase(nn.Module):
    TOPOLOGY = None

    def __init__(self, nc=3, nemb=128, nif=64, use_norm=True, use_spc_norm=False):
        super().__init__()
        self.norm = nn.InstanceNorm2d if use_norm else nn.Identity
        self.nemb = nemb
        mults, k_last = _ENC_TOPOLOGY[self.TOPOLOGY]
        mods, cin = [], nc
        for i, m in enumerate(mults):
            k, s = (3, 1) if i == 0 else (4, 2)
            mods += [spectral_norm(nn.Conv2d(cin, nif * m, k, s, 1, bias=True), use_spc_norm),
                     self.norm(nif * m, affine=True), nn.LeakyReLU(0.2, inplace=True)]
            cin = nif * m
        mods.append(spectral_norm(nn.Conv2d(cin, nemb, k_last, 1, 0), use_spc_norm))
        self.net = nn.Sequential(*mods)

    def forward(self, x):
        # ROCm training forward (grad enabled, x itself not differentiated, as in Q.calculate_loss): libdamc
        # forward + backward (damc.training.encoder_apply) for the shapes it covers
        if x.is_cuda and torch.is_grad_enabled() and not x.requires_grad:
            from damc import training

            if training.ENABLED and training.encoder_train_supported(self, x):
                return training.encoder_apply(self, x)
        return self.net(x).reshape(x.shape[0], self.nemb)


class Encoder_cifar10(_EncoderBase):
    TOPOLOGY = "cifar10"


class Encoder_celeba64(_EncoderBase):
    TOPOLOGY = "celeba64"


class Encoder_celebaHQ(_EncoderBase):
    TOPOLOGY = "celebaHQ"


class Encoder_mnist(_EncoderBase):
    TOPOLOGY = "mnist"

    def __init__(self, nc=1, nemb=128, nif=64, use_norm=True, use_spc_norm=False):
        super().__init__(nc, nemb, nif, use_norm, use_spc_norm)


# -------------------------------------------------------------------------------- denoiser
class ConcatSquashLinearSkipCtx(nn.Module):
    """out = L(x) * sigmoid(Hg(c)) + Hb(c) + S(x), c = SiLU(Lc(SiLU(ctx))) (diffusion_net.py:417-445)."""

    def __init__(self, dim_in, dim_out, nxemb, ntemb, use_spc_norm=False):
        super().__init__()
        self._layer = nn.Sequential(spectral_norm(nn.Linear(dim_in, dim_out), use_spc_norm))
        self._layer_ctx = nn.Sequential(nn.SiLU(), spectral_norm(nn.Linear(ntemb + nxemb, dim_out), use_spc_norm),
                                        nn.SiLU())
        self._hyper_bias = spectral_norm(nn.Linear(dim_out, dim_out, bias=False), use_spc_norm)
        self._hyper_gate = spectral_norm(nn.Linear(dim_out, dim_out), use_spc_norm)
        self._skip = spectral_norm(nn.Linear(dim_in, dim_out), use_spc_norm)

    def forward(self, ctx, x):
        c = self._layer_ctx(ctx)
        return self._layer(x) * torch.sigmoid(self._hyper_gate(c)) + self._hyper_bias(c) + self._skip(x)


class SinusoidalPosEmb(nn.Module):
    """Sinusoidal embedding; scales its input IN PLACE by 1000/max_time like the reference (:447-461)."""

    def __init__(self, dim, max_time=1000.0):
        super().__init__()
        self.dim = dim
        self.max_time = max_time

    _FREQS = {}

    def forward(self, x):
        x *= 1000.0 / self.max_time
        half = self.dim // 2
        # the frequencies by the reference's fp32 ops on the host CPU (its golden path), cached per device: a
        # device's own exp may differ by an ulp, which the ~1000 rad angles below amplify to ~1e-4 in sin / cos
        key = (half, str(x.device))
        freqs = self._FREQS.get(key)
        if freqs is None:
            freqs = torch.exp(torch.arange(half) * (-math.log(10000) / (half - 1))).to(x.device)
            self._FREQS[key] = freqs
        ang = x[:, None] * freqs[None, :]
        if ang.device.type == "cuda":  # sin / cos of the fp32 angle rounded once (the host's libm is within 1 ulp)
            a64 = ang.double()
            return torch.cat((a64.sin(), a64.cos()), dim=-1).to(ang.dtype)
        return torch.cat((ang.sin(), ang.cos()), dim=-1)


class Diffusion_UnetA(nn.Module):
    """U-shaped stack of 7 ConcatSquash blocks over the latent (diffusion_net.py:463-533)."""

    def __init__(self, nz=128, nxemb=128, ntemb=128, residual=False, nf=4):
        super().__init__()
        self.act = F.leaky_relu
        self.nz, self.nxemb, self.ntemb, self.residual = nz, nxemb, ntemb, residual
        self.time_mlp = nn.Sequential(SinusoidalPosEmb(ntemb, max_time=1.0), nn.Linear(ntemb, ntemb), nn.SiLU(),
                                      nn.Linear(ntemb, ntemb))
        self.B = nn.Parameter(data=torch.randn(nz, nz // 2), requires_grad=True)
        w = 32 * nf
        blk = lambda i, o: ConcatSquashLinearSkipCtx(i, o, nxemb, ntemb)  # noqa: E731
        self.in_layers = nn.ModuleList([blk(2 * nz, w), blk(w, 2 * w), blk(2 * w, 2 * w)])
        self.mid_layers = nn.ModuleList([blk(2 * w, 2 * w)])
        self.out_layers = nn.ModuleList([blk(4 * w, 2 * w), blk(4 * w, w), blk(2 * w, nz)])

    def input_emb(self, x):
        proj = 2 * math.pi * (x @ self.B)
        return torch.cat([torch.sin(proj), torch.cos(proj), x], dim=1)

    def forward(self, z, logsnr, xemb):
        b = z.shape[0]
        assert z.shape == (b, self.nz) and logsnr.shape == (b,)
        assert (xemb is None and self.nxemb == 0) or xemb.shape == (b, self.nxemb)
        t_in = torch.arctan(torch.exp(-0.5 * torch.clamp(logsnr, min=-20.0, max=20.0))) / (0.5 * math.pi)
        if z.is_cuda and xemb is not None:
            # ROCm: forward + training backward on libdamc (damc.training.denoiser_apply); the sinusoidal
            # time embedding of the per-sample logsnr stays these torch ops, as the reference evaluates it
            from damc import training

            if training.ENABLED:
                return training.denoiser_apply(self, z, self.time_mlp[0](t_in), xemb)
        temb = self.time_mlp(t_in)
        ctx = temb if xemb is None else torch.cat([temb, xemb], dim=1)
        skips, out = [], self.input_emb(z)
        for layer in self.in_layers:
            out = layer(ctx=ctx, x=out)
            skips.append(out)
            out = self.act(out, negative_slope=0.01)
        out = self.mid_layers[0](ctx=ctx, x=out)
        for layer in self.mid_layers[1:]:
            out = layer(ctx=ctx, x=self.act(out, negative_slope=0.01))
        for layer in self.out_layers:
            out = layer(ctx=ctx, x=self.act(torch.cat([out, skips.pop()], dim=1), negative_slope=0.01))
        assert out.shape == (b, self.nz)
        return z + out if self.residual else out


# ---------------------------------------------------------------------------- amortizer Q
_ENCODER_FOR = {"cifar10": Encoder_cifar10, "svhn": Encoder_cifar10, "mnist": Encoder_mnist,
                "celeba64": Encoder_celeba64}


class _netQ_U(nn.Module):
    """Diffusion-based amortizer: encoder + latent-diffusion reverse sweep (diffusion_net.py:537-645)."""

    def __init__(self, nc=3, nz=128, nxemb=128, ntemb=128, nf=4, nif=64, diffusion_residual=False, n_interval=20,
                 logsnr_min=-20.0, logsnr_max=20.0, var_type="small", with_noise=False, cond_w=0, net_arch="A",
                 dataset="cifar10"):
        super().__init__()
        print("Conditional model Q", with_noise)
        self.n_interval, self.logsnr_min, self.logsnr_max = n_interval, logsnr_min, logsnr_max
        self.var_type, self.nz, self.nxemb, self.with_noise = var_type, nz, nxemb, with_noise
        enc_cls = _ENCODER_FOR.get(dataset, Encoder_celebaHQ)
        self.encoder = enc_cls(nc=1 if dataset == "mnist" else nc, nemb=nxemb, nif=nif)
        self.p = Diffusion_UnetA(nz=nz, nxemb=nxemb, ntemb=ntemb, residual=diffusion_residual, nf=nf)
        self.xemb = nn.Parameter(data=torch.randn(1, self.nxemb), requires_grad=True)
        self.prior_emb = nn.Sequential(nn.Linear(nz, 128), nn.LeakyReLU(), nn.Linear(128, nxemb))
        self.cond_w = cond_w

    def forward(self, x=None, b=None, device=None, cond_w=-1):
        """Reverse sweep on the HIP path (damc.amortizer.q_forward)."""
        from damc import amortizer

        return amortizer.q_forward(self, x=x, b=b, device=device, cond_w=cond_w)

    def _prior_emb(self, noise):
        """self.prior_emb(noise): on ROCm with autograd on, libdamc's forward / backward (damc.training.prior_emb_apply),
        else (or where the C side does not take the shapes) the stock modules."""
        if noise.is_cuda and torch.is_grad_enabled():
            from damc import training

            if training.ENABLED:
                out = training.prior_emb_apply(self.prior_emb, noise)
                if out is not None:
                    return out
        return self.prior_emb(noise)

    def calculate_loss(self, x=None, z=None, mask=None):
        """Training loss of the denoiser (diffusion_net.py:624-645).  On ROCm tensors the denoiser's forward and
        backward run on libdamc (Diffusion_UnetA.forward -> damc.training.denoiser_apply), as do the encoder's
        (_EncoderBase.forward -> damc.training.encoder_apply) and the noising, time embedding and loss
        (damc.training.q_noise_glue / q_loss) and prior_emb (two Linears, used with x None or a mask:
        damc.training.prior_emb_apply); the random draws stay torch's, in the reference's order."""
        assert z is not None
        if x is not None:
            xemb = self.encoder(x)
            if mask is not None:
                xemb = xemb * mask + self._prior_emb(torch.randn(len(x), self.nz, device=x.device)) * (1 - mask)
        else:
            assert mask is None
            xemb = self._prior_emb(torch.randn(len(z), self.nz, device=z.device))
        if z.is_cuda and xemb is not None and not z.requires_grad and z.dtype == torch.float32:
            from damc import training

            if training.ENABLED and training.Q_GLUE:
                # the reference's host-generator draw, copied through pinned memory without blocking: a pageable
                # host-to-device copy waits for the whole stream to drain (tools/h2d_probe.py), which serialised the
                # host's and the GPU's halves of every Q update
                u = training.to_device_async(torch.rand(len(z)), z.device)
                # ROCm: the schedule, the forward diffusion, the time embedding and the loss around the denoiser as
                # libdamc kernels (damc.training.q_noise_glue / q_loss); the draws stay torch's, in the same order
                eps = torch.randn_like(z)
                zt, se = training.q_noise_glue(self, u, z.contiguous(), eps)
                return training.q_loss(eps, training.denoiser_apply(self.p, zt, se, xemb))
        u = torch.rand(len(z)).to(z.device)
        logsnr = logsnr_schedule_fn(u, logsnr_max=self.logsnr_max, logsnr_min=self.logsnr_min)
        fwd = diffusion_forward(z, logsnr=logsnr.reshape(len(z), 1))
        eps = torch.randn_like(z)
        eps_pred = self.p(z=fwd["mean"] + fwd["std"] * eps, logsnr=logsnr, xemb=xemb)
        assert eps.shape == eps_pred.shape == (len(z), self.nz)
        return 0.5 * torch.sum((eps - eps_pred) ** 2, dim=1)
