"""Generator training step on the HIP path.

The G update of a training iteration (workspace/train_gen_recon.py:222-231)::

    x_hat = G(zk_pos)
    g_loss = torch.sum((x_hat - x) ** 2, dim=[1, 2, 3]).mean()
    g_loss.backward()
    G_optimizer.step()

``generator_apply(G, z)`` is what the drop-in ``_netG_*.forward`` runs on ROCm tensors: an autograd
Function whose forward is ``damc_generator_train_forward`` (the Langevin path's generator kernels,
keeping the activations and LReLU' sign bits in a per-call workspace) and whose backward is
``damc_generator_train_backward`` (dL/dx_hat -> every layer's dL/dW, dL/db and optionally dL/dz, with
the k4 s2 p1 / first-layer weight gradients on the limb engine).  The loss, ``clip_grad_norm_`` and the
optimiser stay the caller's PyTorch code, unchanged.  Without grad (``torch.no_grad()``, or nothing
requiring grad) it is the plain HIP forward.
"""
import contextlib
import ctypes
import os
import weakref

import torch

from . import _lib
from ._lib import check, ptr
from .plans import generator_plan

# The drop-in modules route their ROCm training forward/backward here while ENABLED; `stock_pytorch()`
# turns that off explicitly (benchmark comparisons against the reference's own PyTorch path only).
ENABLED = True


@contextlib.contextmanager
def stock_pytorch():
    global ENABLED
    prev, ENABLED = ENABLED, False
    try:
        yield
    finally:
        ENABLED = prev


def _params_of(plan):
    """(layer index, 'w'|'b', parameter) in module order: weight then bias of every layer."""
    out = []
    for i, m in enumerate(plan.modules):
        out.append((i, "w", m.weight))
        if m.bias is not None:
            out.append((i, "b", m.bias))
    return out


class _GeneratorTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, plan, *params):
        dev = z.device
        zc = z.detach().to(torch.float32).contiguous()
        desc = plan.refresh(dev)
        B = zc.shape[0]
        L = _lib.lib()
        nbytes = int(L.damc_generator_train_workspace_bytes(ctypes.byref(desc), B))
        if nbytes == 0:
            raise _lib.DamcError("unsupported generator configuration for the HIP training path")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        shape = (B, plan.nc, plan.h, plan.w) if plan.is_conv else (B, plan.nc)
        xh = torch.empty(shape, dtype=torch.float32, device=dev)
        check(L.damc_generator_train_forward(ctypes.byref(desc), ptr(zc), B, ptr(xh), ptr(ws), nbytes,
                                             _lib.stream_ptr(dev)), "damc_generator_train_forward")
        ctx.plan, ctx.ws, ctx.nbytes = plan, ws, nbytes
        # refresh returned a private descriptor: a later refresh (other engine, other thread) cannot change what
        # the backward runs on — it has to be the engine that filled this workspace
        ctx.desc = desc
        ctx.keep = (plan.buffers, getattr(plan, "_keep", None))
        ctx.save_for_backward(zc, xh, *params)
        return xh

    @staticmethod
    def backward(ctx, gx):
        zc, xh = ctx.saved_tensors[:2]
        if ctx.ws is None:
            raise RuntimeError("the HIP generator backward overwrites its forward's activations as it goes: "
                               "backward through the same G(z) twice (retain_graph=True) is not supported")
        plan = ctx.plan
        dev = zc.device
        # the saved parameters are the modules' own and autograd has checked they were not modified in place,
        # so the packed buffers still hold the forward's weights (any re-pack in between wrote the same
        # values); re-pack only if the plan re-allocated them (device change)
        desc = ctx.desc
        if plan.buffers is not ctx.keep[0]:  # buffers re-allocated (device change): re-pack, same engine
            desc = plan.refresh(dev, engine=desc.layers[0].engine)
        gx = gx.to(torch.float32).contiguous()
        grads = _lib.GeneratorGrads()
        outs = []
        for k, (i, kind, p) in enumerate(_params_of(plan)):
            g = torch.empty_like(p, dtype=torch.float32) if ctx.needs_input_grad[2 + k] else None
            outs.append(g)
            if g is not None:
                getattr(grads, kind)[i] = g.data_ptr()
        gz = torch.empty_like(zc) if ctx.needs_input_grad[0] else None
        check(_lib.lib().damc_generator_train_backward(
            ctypes.byref(desc), ptr(zc), ptr(xh), ptr(gx), zc.shape[0], ctypes.byref(grads), ptr(gz), ptr(ctx.ws),
            ctx.nbytes, _lib.stream_ptr(dev)), "damc_generator_train_backward")
        ctx.ws = ctx.desc = ctx.keep = None
        return (gz, None, *outs)


def generator_apply(G, z):
    """x_hat = G(z) on the HIP path, differentiable w.r.t. z and G's parameters."""
    plan = generator_plan(G)
    if z.dim() == 4:
        z = z.reshape(z.shape[0], -1)
    if z.dim() != 2 or z.shape[1] != plan.nz:
        raise _lib.DamcError("z of shape %s for a generator with nz=%d" % (tuple(z.shape), plan.nz))
    if z.device.type != "cuda":
        raise _lib.DamcError("the HIP generator path needs ROCm tensors (got %s)" % z.device)
    params = [p for _, _, p in _params_of(plan)]
    if torch.is_grad_enabled() and (z.requires_grad or any(p.requires_grad for p in params)):
        return _GeneratorTrainFn.apply(z, plan, *params)
    from .langevin import generator_forward

    return generator_forward(z.to(torch.float32).contiguous(), G)


# ----------------------------------------------------------------------------------------- Q update
# The denoiser of Q.calculate_loss (workspace/src/diffusion_net.py:624-645) on the HIP path
# (SURVEY.md §8f row 2): damc_denoiser_train_forward / _backward over the live parameters in their
# PyTorch layouts (the library stacks them per call).  The encoder / prior_emb / loss stay the caller's
# autograd graph, fed with dL/dxemb.

_BLOCK_KEYS = ("wl", "bl", "ws", "bs", "wg", "bg", "wb", "wctx", "bctx")


def _blocks_of(p):
    return list(p.in_layers) + list(p.mid_layers) + list(p.out_layers)


_DN_PARAMS = weakref.WeakKeyDictionary()  # denoiser -> (entries, owning (module._parameters, name) per entry)


def _denoiser_params(p):
    """[(field, block index or None, parameter)] in a fixed order.  Cached per module (walking ~60 submodule
    attributes costs ~0.1 ms of host time per call, twice per Q update); the cache is revalidated every call against
    the owning modules' parameter dicts, so a parameter replaced by assignment is picked up, and against every
    parent-to-child link of the module tree it walked (a replaced submodule, e.g. ``blk._skip =
    nn.Linear(...)``, leaves the old module's parameter dict intact, so the parameter check alone would hit)."""
    c = _DN_PARAMS.get(p)
    if (c is not None and all(d.get(k) is t for (d, k), (_, _, t) in zip(c[1], c[0])) and
            all(d.get(k) is m for d, k, m in c[2])):
        return c[0]
    links = []

    def child(parent, name):
        m = parent._modules[name]
        links.append((parent._modules, name, m))
        return m

    tm = child(p, "time_mlp")
    t1, t2 = child(tm, "1"), child(tm, "3")
    blocks = []
    for seq in ("in_layers", "mid_layers", "out_layers"):
        ml = child(p, seq)
        blocks += [child(ml, k) for k in list(ml._modules)]
    assert blocks == _blocks_of(p)
    out = [("bmat", None, p.B), ("tw1", None, t1.weight), ("tb1", None, t1.bias), ("tw2", None, t2.weight),
           ("tb2", None, t2.bias)]
    own = [(p._parameters, "B"), (t1._parameters, "weight"), (t1._parameters, "bias"), (t2._parameters, "weight"),
           (t2._parameters, "bias")]
    for b, blk in enumerate(blocks):
        lc = child(child(blk, "_layer_ctx"), "1")
        l0 = child(child(blk, "_layer"), "0")
        sk, hg, hb = child(blk, "_skip"), child(blk, "_hyper_gate"), child(blk, "_hyper_bias")
        mods = (l0, l0, sk, sk, hg, hg, hb, lc, lc)
        names = ("weight", "bias", "weight", "bias", "weight", "bias", "weight", "weight", "bias")
        for key, m, nm in zip(_BLOCK_KEYS, mods, names):
            out.append((key, b, getattr(m, nm)))
            own.append((m._parameters, nm))
    _DN_PARAMS[p] = (out, own, links)
    return out


def _denoiser_desc(p, params):
    d = _lib.DenoiserTrain()
    d.nz, d.ntemb, d.nxemb, d.residual = p.nz, p.ntemb, p.nxemb, int(bool(p.residual))
    for (key, b, _), t in zip(_denoiser_params(p), params):
        if t.dtype != torch.float32 or not t.is_contiguous() or t.device.type != "cuda":
            raise _lib.DamcError("denoiser parameter %s must be a contiguous float32 ROCm tensor" % key)
        if b is None:
            setattr(d, key, t.data_ptr())
        elif key in ("wctx", "bctx"):
            getattr(d, key)[b] = t.data_ptr()
        else:
            setattr(d.blocks[b], key, t.data_ptr())
    for b, blk in enumerate(_blocks_of(p)):
        d.blocks[b].din, d.blocks[b].dout = blk._layer[0].in_features, blk._layer[0].out_features
    return d


def _grad_buffers(params, needed):
    """Gradient tensors for the parameters whose entry of `needed` is set (None elsewhere): contiguous views of ONE
    fp32 allocation, 16-B aligned each (one torch.empty and one split instead of an empty_like per parameter)."""
    sizes, want = [], []
    for p, n in zip(params, needed):
        if n:
            k = p.numel()
            pad = (-k) % 4
            sizes += [k, pad] if pad else [k]
            want.append((p, len(sizes) - (2 if pad else 1)))
        else:
            want.append(None)
    if not want or all(w is None for w in want):
        return [None] * len(want)
    flat = torch.empty(sum(sizes), dtype=torch.float32, device=params[0].device)
    parts = flat.split(sizes)
    return [None if w is None else parts[w[1]].view(w[0].shape) for w in want]


class _DenoiserTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, zt, se, xemb, p, *params):
        dev = zt.device
        zc = zt.detach().to(torch.float32).contiguous()
        sc = se.detach().to(torch.float32).contiguous()
        xc = xemb.detach().to(torch.float32).contiguous()
        desc = _denoiser_desc(p, params)
        B = zc.shape[0]
        L = _lib.lib()
        nbytes = int(L.damc_denoiser_train_workspace_bytes(ctypes.byref(desc), B))
        if nbytes == 0:
            raise _lib.DamcError("unsupported denoiser configuration for the HIP training path")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        eps = torch.empty(B, p.nz, dtype=torch.float32, device=dev)
        check(L.damc_denoiser_train_forward(ctypes.byref(desc), ptr(zc), ptr(sc), ptr(xc), B, ptr(eps), ptr(ws),
                                            nbytes, _lib.stream_ptr(dev)), "damc_denoiser_train_forward")
        ctx.p, ctx.ws, ctx.nbytes, ctx.desc, ctx.B = p, ws, nbytes, desc, B
        ctx.save_for_backward(*params)  # autograd's version check: no in-place update before the backward
        return eps

    @staticmethod
    def backward(ctx, g):
        params = ctx.saved_tensors
        dev = g.device
        g = g.to(torch.float32).contiguous()
        grads = _lib.DenoiserGrads()
        outs = _grad_buffers(params, ctx.needs_input_grad[4:])
        for (key, b, _), t in zip(_denoiser_params(ctx.p), outs):
            if t is not None:
                if b is None:
                    setattr(grads, key, t.data_ptr())
                else:
                    getattr(grads, key)[b] = t.data_ptr()
        gz = torch.empty(ctx.B, ctx.p.nz, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        gx = torch.empty(ctx.B, ctx.p.nxemb, dtype=torch.float32, device=dev) if ctx.needs_input_grad[2] else None
        check(_lib.lib().damc_denoiser_train_backward(
            ctypes.byref(ctx.desc), ptr(g), ctx.B, ctypes.byref(grads), ptr(gz), ptr(gx), ptr(ctx.ws), ctx.nbytes,
            _lib.stream_ptr(dev)), "damc_denoiser_train_backward")
        ctx.ws = ctx.desc = None
        return (gz, None, gx, None, *outs)


def denoiser_apply(p, zt, se, xemb):
    """eps_pred = p(zt, logsnr, xemb) given se = SinusoidalPosEmb(logsnr input), differentiable w.r.t. zt,
    xemb and p's parameters (Diffusion_UnetA.forward, diffusion_net.py:477-533)."""
    params = [t for _, _, t in _denoiser_params(p)]
    return _DenoiserTrainFn.apply(zt, se, xemb, p, *params)


# Q.calculate_loss's noising glue and loss on libdamc (q_noise_glue / q_loss); DAMC_Q_GLUE=0 at import keeps the
# reference's torch ops around the denoiser (A/B)
Q_GLUE = os.environ.get("DAMC_Q_GLUE") != "0"


def to_device_async(t, device):
    """t (a host tensor) on device without blocking the host: through pinned memory (PyTorch's caching host
    allocator keeps the block until the copy has run) with a non-blocking copy; the same values as t.to(device)."""
    if t.device.type != "cpu" or torch.device(device).type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def _freqs(half, device):
    """SinusoidalPosEmb's frequency table, computed as the drop-in computes it (host fp32 ops, then moved)."""
    from src.diffusion_net import SinusoidalPosEmb

    key = (half, str(device))
    f = SinusoidalPosEmb._FREQS.get(key)
    if f is None:
        import math

        f = torch.exp(torch.arange(half) * (-math.log(10000) / (half - 1))).to(device)
        SinusoidalPosEmb._FREQS[key] = f
    return f


def q_noise_glue(q, u, z, eps, logsnr_out=None):
    """(zt, temb_in) of Q.calculate_loss (diffusion_net.py:633-639, 486-491) in one launch (damc_q_noise_glue): the
    schedule's logsnr of u, the forward-diffused zt = mean + std * eps and the denoiser's sinusoidal time embedding.
    No gradient flows through any of it (u and eps are fresh draws; the caller keeps z without grad)."""
    B, nz = z.shape
    ntemb = q.p.ntemb
    dev = z.device
    zt = torch.empty(B, nz, dtype=torch.float32, device=dev)
    se = torch.empty(B, ntemb, dtype=torch.float32, device=dev)
    # the kernel indexes u, z and eps as dense rows; a strided eps (randn_like keeps z's strides) would otherwise be
    # read in its storage order while q_loss reads the logical eps
    u, z, eps = u.contiguous(), z.contiguous(), eps.contiguous()
    check(_lib.lib().damc_q_noise_glue(ptr(u), ptr(z), ptr(eps), B, nz, float(q.logsnr_min), float(q.logsnr_max),
                                       ptr(_freqs(ntemb // 2, dev)), ntemb, ptr(logsnr_out), ptr(zt), ptr(se),
                                       _lib.stream_ptr(dev)), "damc_q_noise_glue")
    return zt, se


class _QLossFn(torch.autograd.Function):
    """0.5 * sum((eps - eps_pred) ** 2, dim=1) (diffusion_net.py:642) as one kernel each way."""

    @staticmethod
    def forward(ctx, eps, pred):
        B, nz = pred.shape
        loss = torch.empty(B, dtype=torch.float32, device=pred.device)
        check(_lib.lib().damc_q_loss_forward(ptr(eps), ptr(pred), B, nz, ptr(loss), _lib.stream_ptr(pred.device)),
              "damc_q_loss_forward")
        ctx.save_for_backward(eps, pred)
        return loss

    @staticmethod
    def backward(ctx, g):
        eps, pred = ctx.saved_tensors
        B, nz = pred.shape
        g = g.to(torch.float32)
        stride = g.stride(0) if g.dim() == 1 else 0
        if g.dim() == 1 and stride != 0 and not g.is_contiguous():
            g, stride = g.contiguous(), 1
        gp = torch.empty_like(pred)
        check(_lib.lib().damc_q_loss_backward(ptr(eps), ptr(pred), ptr(g), stride, B, nz, ptr(gp),
                                              _lib.stream_ptr(pred.device)), "damc_q_loss_backward")
        return None, gp


def q_loss(eps, eps_pred):
    return _QLossFn.apply(eps.contiguous(), eps_pred)


# ----------------------------------------------------------------------------------------- E update
# e_pos, e_neg = E(zk_pos), E(zk_neg); (e_pos.mean() - e_neg.mean()).backward() (train_gen_recon.py:233-241) with
# _netE's forward and backward on libdamc (damc_ebm_train_*): three small-GEMM launches forward, two elementwise and
# two grouped launches backward, instead of ~25 PyTorch ops.  Shapes the C side does not take (batch or widths not a
# multiple of 4, nez != 1, spectral norm, non-fp32 or misaligned tensors) keep the stock PyTorch modules.

def _ebm_layers(E):
    mods = list(E.ebm)
    lins = [m for m in mods if isinstance(m, torch.nn.Linear)]
    acts = [m for m in mods if isinstance(m, torch.nn.LeakyReLU)]
    if len(mods) != 5 or len(lins) != 3 or len(acts) != 2 or mods[0] is not lins[0] or mods[2] is not lins[1]:
        return None
    if any(hasattr(m, "weight_orig") for m in lins) or acts[0].negative_slope != acts[1].negative_slope:
        return None
    # the backward (ebm.hip et_dh2_kernel / et_mask_kernel) reads LReLU' from the sign of the post-activation, which is
    # the pre-activation's sign only for a slope >= 0: other slopes keep the stock modules
    if not acts[0].negative_slope >= 0:
        return None
    if lins[2].out_features != 1 or any(m.bias is None for m in lins):
        return None
    return lins, float(acts[0].negative_slope)


class _EbmTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, desc, slope, *params):
        L = _lib.lib()
        B = z.shape[0]
        nh = desc.nh
        dev = z.device
        h = torch.empty(2, B, nh, dtype=torch.float32, device=dev)
        e = torch.empty(B, dtype=torch.float32, device=dev)
        check(L.damc_ebm_train_forward(ctypes.byref(desc), ptr(z), B, ptr(h[0]), ptr(h[1]), ptr(e),
                                       _lib.stream_ptr(dev)), "damc_ebm_train_forward")
        ctx.desc = desc
        ctx.save_for_backward(z, h, *params)
        return e

    @staticmethod
    def backward(ctx, g):
        z, h = ctx.saved_tensors[:2]
        params = ctx.saved_tensors[2:]
        L = _lib.lib()
        dev = g.device
        B = z.shape[0]
        g = g.to(torch.float32)
        stride = g.stride(0)
        if stride != 0 and not g.is_contiguous():
            g, stride = g.contiguous(), 1
        outs = _grad_buffers(params, ctx.needs_input_grad[3:])
        grads = _lib.EbmGrads()
        for k, t in zip(("w1", "b1", "w2", "b2", "w3", "b3"), outs):
            if t is not None:
                setattr(grads, k, t.data_ptr())
        gz = torch.empty_like(z) if ctx.needs_input_grad[0] else None
        nb = int(L.damc_ebm_train_workspace_bytes(ctypes.byref(ctx.desc), B))
        ws = _scratch("ebm_bwd", dev, nb)
        check(L.damc_ebm_train_backward(ctypes.byref(ctx.desc), ptr(z), ptr(h[0]), ptr(h[1]), ptr(g), stride, B,
                                        ctypes.byref(grads), ptr(gz), ptr(ws), nb, _lib.stream_ptr(dev)),
              "damc_ebm_train_backward")
        ctx.desc = None
        return (gz, None, None, *outs)


def ebm_apply(E, z):
    """E(z).squeeze() on libdamc with grad (the E update), or None where the C side does not take the module / input
    (the caller then runs the stock modules)."""
    lay = _ebm_layers(E)
    if lay is None or z.dim() != 2 or z.dtype != torch.float32 or z.shape[0] % 4:
        return None
    lins, slope = lay
    params = [t for m in lins for t in (m.weight, m.bias)]
    if any(p.dtype != torch.float32 or not p.is_contiguous() or p.data_ptr() % 16 for p in params):
        return None
    z = z.contiguous()
    if z.data_ptr() % 16:
        return None
    d = _lib.Ebm()
    d.nz, d.nh, d.slope = lins[0].in_features, lins[0].out_features, slope
    d.w1, d.b1, d.w2, d.b2, d.w3, d.b3 = [p.data_ptr() for p in params]
    if int(_lib.lib().damc_ebm_train_workspace_bytes(ctypes.byref(d), z.shape[0])) == 0:
        return None
    return _EbmTrainFn.apply(z, d, slope, *params)


# ------------------------------------------------------------------------ Q update: prior embedding
# Q.prior_emb(torch.randn(B, nz)) inside Q.calculate_loss (diffusion_net.py:628-634: the mask's prior rows, or every row
# with x None) on libdamc (damc_prior_emb_train_*): two small-GEMM launches forward, a transpose, two grouped launches
# and the LReLU' mask backward.  Shapes the C side does not take keep the stock modules.

def _prior_emb_layers(seq):
    mods = list(seq)
    if len(mods) != 3 or not isinstance(mods[0], torch.nn.Linear) or not isinstance(mods[2], torch.nn.Linear):
        return None
    if not isinstance(mods[1], torch.nn.LeakyReLU) or not mods[1].negative_slope >= 0:  # LReLU' from h's sign
        return None
    if any(hasattr(m, "weight_orig") or m.bias is None for m in (mods[0], mods[2])):
        return None
    return (mods[0], mods[2]), float(mods[1].negative_slope)


class _PriorEmbTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, noise, desc, *params):
        L = _lib.lib()
        B = noise.shape[0]
        dev = noise.device
        h = torch.empty(B, desc.nh, dtype=torch.float32, device=dev)
        out = torch.empty(B, desc.nout, dtype=torch.float32, device=dev)
        check(L.damc_prior_emb_train_forward(ctypes.byref(desc), ptr(noise), B, ptr(h), ptr(out), _lib.stream_ptr(dev)),
              "damc_prior_emb_train_forward")
        ctx.desc = desc
        ctx.save_for_backward(noise, h, *params)
        return out

    @staticmethod
    def backward(ctx, g):
        noise, h = ctx.saved_tensors[:2]
        params = ctx.saved_tensors[2:]
        L = _lib.lib()
        dev = g.device
        B = noise.shape[0]
        g = g.to(torch.float32).contiguous()
        outs = _grad_buffers(params, ctx.needs_input_grad[2:])
        grads = _lib.PriorEmbGrads()
        for k, t in zip(("w1", "b1", "w2", "b2"), outs):
            if t is not None:
                setattr(grads, k, t.data_ptr())
        nb = int(L.damc_prior_emb_train_workspace_bytes(ctypes.byref(ctx.desc), B))
        ws = _scratch("prior_emb_bwd", dev, nb)
        check(L.damc_prior_emb_train_backward(ctypes.byref(ctx.desc), ptr(noise), ptr(h), ptr(g), B,
                                              ctypes.byref(grads), ptr(ws), nb, _lib.stream_ptr(dev)),
              "damc_prior_emb_train_backward")
        ctx.desc = None
        return (None, None, *outs)


def prior_emb_apply(seq, noise):
    """Q.prior_emb(noise) on libdamc with grad (the Q update), or None where the C side does not take the module /
    input (the caller then runs the stock modules).  noise is a fresh draw: no gradient flows into it."""
    lay = _prior_emb_layers(seq)
    if lay is None or noise.dim() != 2 or noise.dtype != torch.float32 or noise.shape[0] % 4 or noise.requires_grad:
        return None
    (l1, l2), slope = lay
    params = [l1.weight, l1.bias, l2.weight, l2.bias]
    if any(p.dtype != torch.float32 or not p.is_contiguous() or p.device != noise.device or p.data_ptr() % 16
           for p in params):
        return None
    noise = noise.contiguous()
    if noise.data_ptr() % 16:
        return None
    d = _lib.PriorEmb()
    d.nz, d.nh, d.nout, d.slope = l1.in_features, l1.out_features, l2.out_features, slope
    d.w1, d.b1, d.w2, d.b2 = [p.data_ptr() for p in params]
    if l2.in_features != d.nh or int(_lib.lib().damc_prior_emb_train_workspace_bytes(ctypes.byref(d), noise.shape[0])) == 0:
        return None
    return _PriorEmbTrainFn.apply(noise, d, *params)


# ------------------------------------------------------------------------------- Q update: encoder
# Encoder_* (workspace/src/diffusion_net.py:227-413) as trained by Q.calculate_loss: forward on libdamc
# keeping every conv output, InstanceNorm statistic and layer input; backward through
# damc_instnorm_lrelu_backward_nhwc and damc_conv2d_backward_nhwc (the generator's limb-engine kernels with the
# roles swapped for the k4 s2 p1 convs).  Shapes the C side does not cover keep the stock PyTorch path
# (encoder_train_supported is False for them; the Q-update tests assert which path ran).

_ENC_SUPPORT = weakref.WeakKeyDictionary()  # encoder -> {input shape: verdict}; dies with the encoder


def _enc_stages(enc):
    from .amortizer import EncoderPlan

    return EncoderPlan(enc).stages


def _enc_params(stages):
    out = []
    for conv, norm, _ in stages:
        out += [conv.weight, conv.bias]
        if norm is not None:
            out += [norm.weight, norm.bias]
    return out


def encoder_train_supported(enc, x):
    per_enc = _ENC_SUPPORT.setdefault(enc, {})
    key = tuple(x.shape)
    hit = per_enc.get(key)
    if hit is not None:
        return hit
    ok = True
    try:
        stages = _enc_stages(enc)
        B, _, H, W = x.shape
        L = _lib.lib()
        for i, (conv, norm, _) in enumerate(stages):
            k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            if conv.bias is None or (norm is None) != (i == len(stages) - 1):
                ok = False
                break
            if int(L.damc_conv2d_backward_workspace_bytes(B, H, W, conv.in_channels, conv.out_channels, k, s, p)) == 0:
                ok = False
                break
            H, W = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        ok = ok and H == 1 and W == 1
    except NotImplementedError:
        ok = False
    per_enc[key] = ok
    return ok


# per-call scratch of the encoder's training forward / backward (packed weights, conv and InstanceNorm workspaces):
# kernels are stream-ordered, so one buffer per purpose serves every stage and every call on a stream (round 5: ~20
# torch.empty calls per Q update, ~0.1 ms of host time)
_ENC_SCRATCH = {k: _lib.WorkspaceCache() for k in ("w3", "conv", "in", "in_bwd", "conv_bwd", "ebm_bwd", "enc_train", "prior_emb_bwd")}


def _scratch(key, device, nbytes):
    return _ENC_SCRATCH[key].get(device, max(int(nbytes), 16), key)


class _EncoderTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, stages, *params):
        L = _lib.lib()
        dev = x.device
        stream = _lib.stream_ptr(dev)
        B, C, H, W = x.shape
        h = torch.empty(B, H, W, C, dtype=torch.float32, device=dev)
        check(L.damc_nchw_to_nhwc(ptr(x.detach().float().contiguous()), B, C, H * W, ptr(h), stream), "nchw_to_nhwc")
        saved = []
        limb = _lib.current_engine() == _lib.ENGINE_LIMB
        for conv, norm, slope in stages:
            k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            cout, cin = conv.out_channels, conv.in_channels
            Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
            y = torch.empty(B, Ho, Wo, cout, dtype=torch.float32, device=dev)
            nbx = int(L.damc_conv2d_x3_workspace_bytes(B, H, W, cin, cout, k, s, p)) if limb else 0
            if nbx:  # the limb engine (fp32-accurate bf16 MFMA), as the Q(x) forward runs these convs (a10)
                w3 = _scratch("w3", dev, L.damc_conv2d_x3_bytes(cout, cin, k))
                check(L.damc_pack_conv2d_x3(ptr(conv.weight.detach().contiguous()), cout, cin, k, ptr(w3), stream),
                      "pack conv2d x3")
                ws = _scratch("conv", dev, nbx)
                check(L.damc_conv2d_x3_nhwc(ptr(h), B, H, W, cin, ptr(w3), ptr(conv.bias), cout, k, s, p, ptr(y),
                                            ptr(ws), nbx, stream), "conv2d x3")
            else:
                wp = torch.empty(k * k * cin * cout, dtype=torch.float32, device=dev)
                check(L.damc_pack_conv2d(ptr(conv.weight), cout, cin, k, ptr(wp), stream), "pack conv2d")
                nsl = int(L.damc_conv2d_workspace_floats(B, H, W, cin, cout, k, s, p))
                sl = torch.empty(nsl, dtype=torch.float32, device=dev) if nsl else None
                check(L.damc_conv2d_nhwc(ptr(h), B, H, W, cin, ptr(wp), ptr(conv.bias), cout, k, s, p, ptr(y),
                                         ptr(sl), nsl, stream), "conv2d")
            stats, out = None, y
            if norm is not None:
                out = torch.empty_like(y)
                stats = torch.empty(B * cout * 2, dtype=torch.float32, device=dev)
                ws = _scratch("in", dev, 4 * int(L.damc_instnorm_workspace_floats(B, Ho * Wo, cout)))
                check(L.damc_instnorm_lrelu_train_nhwc(ptr(y), B, Ho * Wo, cout, ptr(norm.weight), ptr(norm.bias),
                                                       float(norm.eps), float(slope), ptr(out), ptr(stats), ptr(ws),
                                                       stream), "instnorm train")
            saved.append((h, y, stats, H, W, Ho, Wo))
            h, H, W = out, Ho, Wo
        ctx.stages, ctx.saved, ctx.B = stages, saved, B
        ctx.save_for_backward(*params)
        return h.reshape(B, -1)

    @staticmethod
    def backward(ctx, g):
        L = _lib.lib()
        dev = g.device
        stream = _lib.stream_ptr(dev)
        B = ctx.B
        params = ctx.saved_tensors
        grads = _grad_buffers(params, ctx.needs_input_grad[2:])
        # parameter index of each stage's (conv.weight, conv.bias, norm.weight, norm.bias)
        idx, pos = [], 0
        for conv, norm, _ in ctx.stages:
            idx.append(pos)
            pos += 4 if norm is not None else 2
        dh = g.to(torch.float32).contiguous()
        for i in range(len(ctx.stages) - 1, -1, -1):
            conv, norm, slope = ctx.stages[i]
            h_in, y, stats, H, W, Ho, Wo = ctx.saved[i]
            k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
            cout, cin = conv.out_channels, conv.in_channels
            j = idx[i]
            if norm is not None:
                dy = torch.empty_like(y)
                ws = _scratch("in_bwd", dev, 4 * int(L.damc_instnorm_bwd_workspace_floats(B, Ho * Wo, cout)))
                check(L.damc_instnorm_lrelu_backward_nhwc(ptr(y), ptr(stats), ptr(dh), B, Ho * Wo, cout,
                                                          ptr(norm.weight), ptr(norm.bias), float(slope), ptr(dy),
                                                          ptr(grads[j + 2]), ptr(grads[j + 3]), ptr(ws), stream),
                      "instnorm backward")
            else:
                dy = dh
            dx = torch.empty(B, H, W, cin, dtype=torch.float32, device=dev) if i > 0 else None
            nbytes = int(L.damc_conv2d_backward_workspace_bytes(B, H, W, cin, cout, k, s, p))
            ws = _scratch("conv_bwd", dev, nbytes)
            dw = grads[j] if grads[j] is not None else torch.empty_like(conv.weight)
            check(L.damc_conv2d_backward_nhwc(ptr(h_in), ptr(dy), ptr(conv.weight), B, H, W, cin, cout, k, s, p,
                                              ptr(dx), ptr(dw), ptr(grads[j + 1]), ptr(ws), nbytes, stream),
                  "conv2d backward")
            dh = dx
        ctx.saved = None
        return (None, None, *grads)


# round 5: the whole encoder in one library call each way (damc_encoder_train_forward / _backward) instead of ~4 calls
# per stage from Python; DAMC_ENC_TRAIN_FUSED=0 (read at import) keeps the per-stage Function above
ENC_TRAIN_FUSED = os.environ.get("DAMC_ENC_TRAIN_FUSED") != "0"
_ENC_DESC = weakref.WeakKeyDictionary()  # encoder -> (key of parameter pointers and input shape, descriptor, sizes)


def _enc_train_desc(enc, stages, params, x):
    """The damc_encoder_t of the training calls, cached per encoder while its parameters' storage and the input
    shape stay the same (the descriptor holds raw pointers, read by the library at each call)."""
    key = (tuple(p.data_ptr() for p in params), tuple(x.shape), _lib.current_engine())
    c = _ENC_DESC.get(enc)
    if c is not None and c[0] == key:
        return c[1], c[2], c[3]
    d = _lib.Encoder()
    B, C, H, W = x.shape
    d.n_layers, d.nc, d.h, d.w = len(stages), C, H, W
    d.engine = _lib.current_engine()
    for i, (conv, norm, slope) in enumerate(stages):
        L = d.layers[i]
        L.cin, L.cout, L.k = conv.in_channels, conv.out_channels, conv.kernel_size[0]
        L.stride, L.pad = conv.stride[0], conv.padding[0]
        L.w_src, L.bias = conv.weight.data_ptr(), conv.bias.data_ptr()
        if norm is not None:
            L.in_gamma, L.in_beta, L.in_eps = norm.weight.data_ptr(), norm.bias.data_ptr(), float(norm.eps)
        L.slope = float(slope) if slope is not None else 0.0
    lib = _lib.lib()
    nsaved = int(lib.damc_encoder_train_saved_floats(ctypes.byref(d), B))
    nws = int(lib.damc_encoder_train_workspace_bytes(ctypes.byref(d), B))
    _ENC_DESC[enc] = (key, d, nsaved, nws)
    return d, nsaved, nws


class _EncoderTrainFusedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, enc, stages, *params):
        L = _lib.lib()
        dev = x.device
        xc = x.detach().float().contiguous()
        d, nsaved, nws = _enc_train_desc(enc, stages, params, xc)
        if nsaved == 0 or nws == 0:
            raise _lib.DamcError("encoder configuration not supported by damc_encoder_train_forward")
        B = xc.shape[0]
        saved = torch.empty(nsaved, dtype=torch.float32, device=dev)
        xemb = torch.empty(B, stages[-1][0].out_channels, dtype=torch.float32, device=dev)
        check(L.damc_encoder_train_forward(ctypes.byref(d), ptr(xc), B, ptr(saved), ptr(xemb),
                                           ptr(_scratch("enc_train", dev, nws)), nws, _lib.stream_ptr(dev)),
              "damc_encoder_train_forward")
        ctx.d, ctx.nws, ctx.saved_buf, ctx.B = d, nws, saved, B
        ctx.save_for_backward(*params)  # autograd's version check: no in-place update before the backward
        return xemb

    @staticmethod
    def backward(ctx, g):
        L = _lib.lib()
        dev = g.device
        params = ctx.saved_tensors
        grads = _grad_buffers(params, ctx.needs_input_grad[3:])
        gs = _lib.EncoderGrads()
        j = 0
        for i in range(ctx.d.n_layers):
            has_norm = bool(ctx.d.layers[i].in_gamma)
            gs.w[i] = None if grads[j] is None else grads[j].data_ptr()
            gs.b[i] = None if grads[j + 1] is None else grads[j + 1].data_ptr()
            if has_norm:
                gs.gamma[i] = None if grads[j + 2] is None else grads[j + 2].data_ptr()
                gs.beta[i] = None if grads[j + 3] is None else grads[j + 3].data_ptr()
                j += 4
            else:
                j += 2
        g = g.to(torch.float32).contiguous()
        check(L.damc_encoder_train_backward(ctypes.byref(ctx.d), ptr(ctx.saved_buf), ptr(g), ctx.B, ctypes.byref(gs),
                                            ptr(_scratch("enc_train", dev, ctx.nws)), ctx.nws, _lib.stream_ptr(dev)),
              "damc_encoder_train_backward")
        ctx.saved_buf = ctx.d = None
        return (None, None, None, *grads)


def encoder_apply(enc, x):
    """xemb = Encoder_*(x) on the HIP path, differentiable w.r.t. the encoder's parameters (not x)."""
    stages = _enc_stages(enc)
    params = _enc_params(stages)
    if ENC_TRAIN_FUSED:
        return _EncoderTrainFusedFn.apply(x, enc, stages, *params)
    return _EncoderTrainFn.apply(x, stages, *params)
