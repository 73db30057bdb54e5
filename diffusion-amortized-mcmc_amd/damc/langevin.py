"""Tensor-level Langevin API over libdamc (the functions behind src/MCMC.py).

All functions run on the caller's current HIP stream, never synchronise the host (unless a
diagnostics tensor is read by the caller), and update ``z`` in place.

Noise: ``noise=None`` with ``with_noise`` draws xi in-kernel (Philox4x32-10) keyed by ``seed``
and the chain's GLOBAL index ``chain_base + row`` and step ``step_offset + i``; passing
``noise`` (n_steps, B, nz) injects values instead (parity tests).

Spectral-norm nets in train mode (nn.utils.spectral_norm, diffusion_net.py:8-16): every forward of the reference
advances each layer's u, v by one power iteration, so the weights change from step to step.  The chains then run one
step per library call, each after that step's power iterations (plans.spectral_norm_step) and a re-pack; the noise is
the same Philox stream (keyed by step_offset + i), so a chain keeps its values whichever way it is cut.
"""
import ctypes

import torch

from . import _lib
from ._lib import check, ptr
from .plans import ebm_plan, generator_plan, spectral_norm_step


def _f32c(t, name):
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise _lib.DamcError("%s must be a contiguous float32 tensor" % name)
    if t.device.type != "cuda":
        raise _lib.DamcError("%s must be on a ROCm device (got %s); the HIP path has no CPU fallback" % (name, t.device))
    return t


def new_seed():
    """A Philox key drawn from torch's (seeded) CPU generator."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def posterior_langevin(z, x, netG, netE, n_steps, sigma, step, with_noise, noise=None, seed=None,
                       step_offset=0, chain_base=0, diag=False):
    """In-place n-step posterior Langevin (workspace/src/MCMC.py:48-74) on z (B, nz).

    Returns a (n_steps, 4) diagnostics tensor {sum E, lik, |z|^2/2, mean grad} if diag else None.
    """
    _f32c(z, "z")
    dev = z.device
    x = x.to(device=dev, dtype=torch.float32).contiguous()
    B = z.shape[0]
    gp = generator_plan(netG)
    if z.shape[1] != gp.nz or x.shape[0] != B or x.numel() != B * gp.nc * gp.h * gp.w:
        raise _lib.DamcError("shape mismatch: z %s x %s for generator nz=%d out=(%d,%d,%d)"
                             % (tuple(z.shape), tuple(x.shape), gp.nz, gp.nc, gp.h, gp.w))
    ep = ebm_plan(netE) if netE is not None else None
    if noise is not None:
        noise = _f32c(noise.to(dev), "noise")
        if noise.numel() < n_steps * B * gp.nz:
            raise _lib.DamcError("noise must hold (n_steps, B, nz) values")
    if seed is None:
        seed = new_seed() if (with_noise and noise is None) else 0
    dg = torch.zeros(max(n_steps, 1), 4, dtype=torch.float32, device=dev) if diag else None

    def run(n, off, nz_, dg_):
        gdesc = gp.refresh(dev)
        edesc = ep.refresh(dev) if ep is not None else None
        ws, nbytes = gp.workspace(B)
        check(_lib.lib().damc_posterior_langevin(
            ctypes.byref(gdesc), ctypes.byref(edesc) if edesc is not None else None, ptr(z), ptr(x), B, int(n),
            float(sigma), float(step), int(bool(with_noise)), ptr(nz_), seed, off, chain_base,
            ptr(dg_), ptr(ws), nbytes, _lib.stream_ptr(dev)), "damc_posterior_langevin")

    sn = gp.sn_train() + (ep.sn_train() if ep is not None else [])
    if not sn:
        run(n_steps, step_offset, noise, dg)
        return dg
    # train-mode spectral norm: netG(z) and netE(z) once per reference step (MCMC.py:54-58), one power iteration each
    nzs = noise.view(-1, B * gp.nz) if noise is not None else None
    for i in range(int(n_steps)):
        with spectral_norm_step(sn):
            run(1, step_offset + i, nzs[i] if nzs is not None else None, dg[i] if dg is not None else None)
    return dg


def likelihood_grad(z, x, netG, sigma):
    """grad_z |G(z)-x|^2/(2 sigma^2) (per-op hook)."""
    _f32c(z, "z")
    dev = z.device
    x = x.to(device=dev, dtype=torch.float32).contiguous()
    gp = generator_plan(netG)
    with spectral_norm_step(gp.sn_train()):  # one G forward (train-mode spectral norm: one power iteration)
        gdesc = gp.refresh(dev)
    ws, nbytes = gp.workspace(z.shape[0])
    g = torch.empty_like(z)
    check(_lib.lib().damc_likelihood_grad(ctypes.byref(gdesc), ptr(z), ptr(x), z.shape[0], float(sigma), ptr(g),
                                          ptr(ws), nbytes, _lib.stream_ptr(dev)), "damc_likelihood_grad")
    return g


def generator_forward(z, netG):
    """x_hat = G(z) on the HIP path (NCHW, or (B, out) for MLP generators)."""
    z = _f32c(z.detach().contiguous() if not z.is_contiguous() else z.detach(), "z")
    dev = z.device
    gp = generator_plan(netG)
    with spectral_norm_step(gp.sn_train()):  # one G forward (train-mode spectral norm: one power iteration)
        gdesc = gp.refresh(dev)
    ws, nbytes = gp.workspace(z.shape[0])
    shape = (z.shape[0], gp.nc, gp.h, gp.w) if gp.is_conv else (z.shape[0], gp.nc)
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    check(_lib.lib().damc_generator_forward(ctypes.byref(gdesc), ptr(z), z.shape[0], ptr(out), ptr(ws), nbytes,
                                            _lib.stream_ptr(dev)), "damc_generator_forward")
    return out


PRIOR_ENGINES = {"auto": 0, "valu": 1, "mfma": 2}


def mfma_min_chains():
    """Chain count from which "auto" picks the MFMA prior engine: the library's own threshold
    (DAMC_EBM_MFMA_MIN_B read once per process), so Python and a C caller of engine 0 always agree."""
    return int(_lib.lib().damc_ebm_mfma_min_chains())


def prior_langevin(z, netE, n_steps, step, with_noise, noise=None, seed=None, step_offset=0, chain_base=0,
                   diag=False, engine="auto", global_batch=None):
    """In-place n-step prior Langevin (workspace/src/MCMC.py:27-46), one persistent launch.

    engine: "auto" (by chain count), "valu" (one chain per workgroup, weights in registers) or "mfma" (16-chain
    tiles on the fp32 MFMA).  The two engines sum in different orders, so "auto" decides from ``global_batch``
    (the chain count of the whole sharded block; default: this call's) — every shard of a block then runs the
    engine the unsharded block runs, and the union of the shards stays bitwise the one-GPU result.  Returns a
    (n_steps, 2) diagnostics tensor {sum E, |z|^2/2} if diag else None.
    """
    _f32c(z, "z")
    dev = z.device
    ep = ebm_plan(netE)
    if z.shape[1] != ep.nz:
        raise _lib.DamcError("z has %d dims, EBM expects %d" % (z.shape[1], ep.nz))
    B = z.shape[0]
    if noise is not None:
        noise = _f32c(noise.to(dev), "noise")
        if noise.numel() < n_steps * B * ep.nz:
            raise _lib.DamcError("noise must hold (n_steps, B, nz) values")
    if seed is None:
        seed = new_seed() if (with_noise and noise is None) else 0
    dg = torch.zeros(max(n_steps, 1), 2, dtype=torch.float32, device=dev) if diag else None
    if engine not in PRIOR_ENGINES:
        raise ValueError("engine must be one of %s" % sorted(PRIOR_ENGINES))
    code = PRIOR_ENGINES[engine]
    if engine == "auto":  # resolved here from the global chain count, never from the shard's
        code = 2 if int(global_batch if global_batch is not None else B) >= mfma_min_chains() else 1

    def run(n, off, nz_, dg_):
        edesc = ep.refresh(dev)

        def call(c):
            return _lib.lib().damc_prior_langevin_engine(ctypes.byref(edesc), ptr(z), B, int(n), float(step),
                                                         int(bool(with_noise)), ptr(nz_), seed, off,
                                                         chain_base, ptr(dg_), c, _lib.stream_ptr(dev))

        rc = call(code)
        if rc == _lib.DAMC_ERR_UNSUPPORTED and engine == "auto":  # the shape has no kernel of that engine: the other
            rc = call(1 if code == 2 else 2)
        check(rc, "damc_prior_langevin")

    sn = ep.sn_train()
    if not sn:
        run(n_steps, step_offset, noise, dg)
        return dg
    # train-mode spectral norm: netE(z) once per reference step (MCMC.py:32), one power iteration each
    nzs = noise.view(-1, B * ep.nz) if noise is not None else None
    for i in range(int(n_steps)):
        with spectral_norm_step(sn):
            run(1, step_offset + i, nzs[i] if nzs is not None else None, dg[i] if dg is not None else None)
    return dg


def ebm_energy_grad(z, netE):
    _f32c(z, "z")
    dev = z.device
    ep = ebm_plan(netE)
    with spectral_norm_step(ep.sn_train()):  # one E forward (train-mode spectral norm: one power iteration)
        edesc = ep.refresh(dev)
    e = torch.empty(z.shape[0], dtype=torch.float32, device=dev)
    g = torch.empty_like(z)
    check(_lib.lib().damc_ebm_energy_grad(ctypes.byref(edesc), ptr(z), z.shape[0], ptr(e), ptr(g),
                                          _lib.stream_ptr(dev)), "damc_ebm_energy_grad")
    return e, g


def philox_normal(n_steps, batch, nz, seed, device, step_offset=0, chain_base=0, stream_id=0x51):
    out = torch.empty(n_steps, batch, nz, dtype=torch.float32, device=device)
    check(_lib.lib().damc_philox_normal(ptr(out), n_steps, batch, nz, seed, step_offset, chain_base, stream_id,
                                        _lib.stream_ptr(device)), "damc_philox_normal")
    return out


def z_update(z, g, step, with_noise, noise=None, seed=0, step_index=0, chain_base=0):
    """Per-op hook: z <- z - 0.5 step^2 (g + z) (+ step xi), in place (MCMC.py:36-38,62-64)."""
    _f32c(z, "z")
    _f32c(g, "g")
    if g.shape != z.shape:
        raise _lib.DamcError("g must have z's shape")
    if noise is not None:
        noise = _f32c(noise, "noise")
        if noise.numel() < z.numel():
            raise _lib.DamcError("noise must hold (B, nz) values")
    check(_lib.lib().damc_z_update(ptr(z), ptr(g), z.shape[0], z.shape[1], float(step), int(bool(with_noise)),
                                   ptr(noise), seed, step_index, chain_base, _lib.stream_ptr(z.device)),
          "damc_z_update")
    return z
