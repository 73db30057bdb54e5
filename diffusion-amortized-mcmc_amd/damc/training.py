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
import ctypes

import torch

from . import _lib
from ._lib import check, ptr
from .plans import generator_plan


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
        ctx.desc, ctx.keep = desc, (plan.buffers, getattr(plan, "_keep", None))
        ctx.save_for_backward(zc, xh, *params)
        return xh

    @staticmethod
    def backward(ctx, gx):
        zc, xh = ctx.saved_tensors[:2]
        plan = ctx.plan
        dev = zc.device
        # the saved parameters are the modules' own and autograd has checked they were not modified in place,
        # so the packed buffers still hold the forward's weights (any re-pack in between wrote the same
        # values); re-pack only if the plan re-allocated them (device change)
        desc = ctx.desc if plan.desc is ctx.desc else plan.refresh(dev)
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
