"""clip_grad_norm_ + Adam / AdamW on the HIP optimiser kernels ("a fused Adam step").

The reference trains G with ``optim.Adam(betas=(0.5, 0.999))``, Q with ``optim.AdamW(weight_decay=1e-4)`` and
E with ``optim.Adam`` (``workspace/train_gen_recon.py:155-157``), each step preceded by
``torch.nn.utils.clip_grad_norm_`` (``:219``, ``:230``, ``:240``).  ``Adam`` / ``AdamW`` here are
``torch.optim.Optimizer`` subclasses with the same constructor, ``param_groups`` defaults and per-parameter
state (``step`` fp32 CPU scalar, ``exp_avg``, ``exp_avg_sq``), so ``state_dict()`` / ``load_state_dict()``
interchange with torch's (the reference checkpoints its optimisers, ``train_gen_recon.py:284-294``).

``step()`` is one ``damc_adam_step`` launch per 96 parameters of a group (``csrc/optim.hip``: one pass reading
p, g, m, v and writing p, m, v, in torch's ``_multi_tensor_adam`` op order).  The tensors' device pointers go
in the kernel arguments; the only device-side table (chunk -> tensor, offset, length) depends on the sizes
alone and is built once.  ``clip_grad_norm_`` is the deterministic HIP norm plus a scaling pass, returning
the total norm like torch's.  ``clip_and_step(max_norm)`` fuses the two: the norm pass, then the Adam pass
applies the clip factor (and leaves the gradients scaled, as ``clip_grad_norm_`` would have).  There is no
fallback: CPU tensors, non-fp32 or non-contiguous tensors, and the unsupported flags (amsgrad, maximize,
capturable, differentiable, tensor lr) raise.
"""
import ctypes

import torch

from . import _lib

MAXT = _lib.ADAM_MAX_TENSORS
_CHUNK_BYTES = 16  # sizeof(AdamChunk), checked against the library on first use
_VP = ctypes.c_void_p


def _check(code, what):
    if code != 0:
        raise _lib.DamcError("%s failed: %s" % (what, _lib.lib().damc_error_string(code).decode()))


def _require_fp32_cuda(t, what):
    if not t.is_cuda:
        raise _lib.DamcError("%s: damc.optim runs on the HIP kernels only (got a %s tensor)" % (what, t.device))
    if t.dtype != torch.float32 or t.is_sparse or not t.is_contiguous():
        raise _lib.DamcError("%s: needs dense contiguous float32 tensors" % what)


class _Chunks:
    """Chunk tables of a list of tensor sizes, one per <= MAXT-tensor slice: [(t0, t1, dev, n, base)]."""

    _cache = {}

    @classmethod
    def of(cls, numels, device):
        key = (str(device), tuple(numels))
        c = cls._cache.get(key)
        if c is None:
            if len(cls._cache) > 64:
                cls._cache.clear()
            c = cls._cache[key] = cls(numels, device)
        return c

    def __init__(self, numels, device):
        L = _lib.lib()
        if L.damc_adam_chunk_bytes() != _CHUNK_BYTES:
            raise _lib.DamcError("libdamc AdamChunk layout mismatch")
        self.slices, base = [], 0
        for t0 in range(0, len(numels), MAXT):
            ns = numels[t0:t0 + MAXT]
            arr = (ctypes.c_longlong * len(ns))(*ns)
            cnt = L.damc_adam_chunk_count(arr, len(ns))
            if cnt < 0:
                raise _lib.DamcError("damc_adam_chunk_count failed (%d)" % cnt)
            host = (ctypes.c_ubyte * (_CHUNK_BYTES * max(cnt, 1)))()
            k = L.damc_adam_build_chunks(arr, len(ns), host, cnt)
            if k < 0:
                raise _lib.DamcError("damc_adam_build_chunks failed (%d)" % k)
            dev = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(device)
            self.slices.append((t0, t0 + len(ns), dev, k, base))
            base += k
        self.nchunks = base
        self.partial = torch.empty(max(base, 1), dtype=torch.float32, device=device)


def _ptrs(ts):
    return (_VP * len(ts))(*[t.data_ptr() for t in ts])


def _stream():
    return _VP(torch.cuda.current_stream().cuda_stream)


def _norm(chunks, grads, max_norm):
    """clip_grad_norm_'s total norm and clip factor: out = [norm, min(max_norm / (norm + 1e-6), 1)]."""
    L = _lib.lib()
    out = torch.empty(2, dtype=torch.float32, device=grads[0].device)
    s = _stream()
    for t0, t1, dev, n, base in chunks.slices:
        _check(L.damc_grad_sumsq(_VP(dev.data_ptr()), n, _ptrs(grads[t0:t1]), t1 - t0,
                                 _VP(chunks.partial.data_ptr() + 4 * base), s), "damc_grad_sumsq")
    _check(L.damc_grad_norm_finish(_VP(chunks.partial.data_ptr()), chunks.nchunks, float(max_norm),
                                   _VP(out.data_ptr()), s), "damc_grad_norm_finish")
    return out


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam on ``damc_adam_step`` (same arguments; see the module docstring for the limits)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=False, differentiable=False, fused=None,
                 decoupled_weight_decay=False):
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("damc.optim.Adam: amsgrad / maximize / capturable / differentiable")
        if isinstance(lr, torch.Tensor) or any(isinstance(b, torch.Tensor) for b in betas):
            raise NotImplementedError("damc.optim.Adam: tensor lr / betas")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError("invalid Adam hyper-parameters")
        if not 0.0 <= weight_decay:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused,
                        decoupled_weight_decay=decoupled_weight_decay)
        super().__init__(params, defaults)
        self.last_grad_norm = None

    def __setstate__(self, state):
        super().__setstate__(state)
        self.last_grad_norm = None

    def state_dict(self):
        """torch.optim.Optimizer.state_dict with a private ``step`` tensor per parameter.  ``_advance_steps`` lets the
        parameters of a group share one counter; torch's own state_dict (and torch.save / torch.load after it) would
        keep that sharing, and a stock Adam / AdamW that loads it adds 1 to the shared tensor once per parameter
        (every count 6.0 instead of 3.0 after one resumed step).  The clones carry the same values, so the
        dict interchanges with torch's; this optimiser's own state keeps the shared counter."""
        sd = super().state_dict()
        sd["state"] = {k: ({**v, "step": v["step"].clone()} if isinstance(v.get("step"), torch.Tensor) else v)
                       for k, v in sd["state"].items()}
        return sd

    def zero_grad(self, set_to_none=True):
        """torch.optim.Optimizer.zero_grad; set_to_none (the default) as a plain loop (torch's walks the same
        parameters through its profiler scope and foreach grouping: ~0.1 ms of host time per Q update)."""
        if not set_to_none:
            return super().zero_grad(set_to_none=False)
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

    def _collect(self, group):
        """(params, grads, exp_avgs, exp_avg_sqs, steps) of the group's parameters that have a gradient."""
        ps, gs, ms, vs, steps = [], [], [], [], []
        f32, strided = torch.float32, torch.strided
        for p in group["params"]:
            g = p.grad
            if g is None:
                continue
            # _require_fp32_cuda on both, one expression on the common case (the checks themselves were ~0.1 ms per
            # 100-parameter step)
            if not (p.dtype is f32 and g.dtype is f32 and p.is_cuda and g.is_cuda and p.layout is strided and
                    g.layout is strided and p.is_contiguous() and g.is_contiguous()):
                _require_fp32_cuda(p, "param")
                _require_fp32_cuda(g, "grad")
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            ps.append(p)
            gs.append(g)
            ms.append(st["exp_avg"])
            vs.append(st["exp_avg_sq"])
            steps.append(st["step"])
        return ps, gs, ms, vs, steps

    def _advance_steps(self, group, steps):
        """+1 on the step counters of the parameters being updated, as torch's _multi_tensor_adam does, and their
        common value (None when they differ).  Where every parameter of the group is updated and all counters agree,
        the group's states share ONE step tensor (equal values, so torch's state_dict and load_state_dict see the
        same counts), and the advance is one add instead of a foreach over ~100 CPU scalars plus a stack and a
        compare (~0.6 ms of host time per Q update)."""
        shared = steps[0]
        if all(t is shared for t in steps):
            # one counter for every updated parameter: advance it once, unless a parameter left out of this step
            # (no gradient) holds it too.  Round 5: the Q update leaves some of Q's parameters without a gradient
            # every step, which sent each step through the per-parameter path below (~0.3 ms of host time)
            partial = len(steps) < len(group["params"])
            if not partial or not any((self.state.get(p) or {}).get("step") is shared
                                      for p in group["params"] if p.grad is None):
                shared.add_(1.0)
                return float(shared)
        if len(steps) < len(group["params"]) or len({id(t) for t in steps}) < len(steps):
            # a shared counter and only some parameters updated: each updated parameter gets its own counter first
            i = 0
            for p in group["params"]:
                if p.grad is None:
                    continue
                steps[i] = self.state[p]["step"] = steps[i].clone()
                i += 1
        torch._foreach_add_(steps, 1.0)
        sv = torch.stack(steps)
        if not bool((sv == sv[0]).all()):
            return None
        # the updated parameters agree: they share one counter from here on (private to them: the partial path above
        # gave each its own copy first)
        one = steps[0]
        for p in group["params"]:
            if p.grad is not None:
                self.state[p]["step"] = one
        return float(sv[0])

    @staticmethod
    def _hparams(group, step):
        beta1, beta2 = group["betas"]
        lr, wd = group["lr"], group["weight_decay"]
        h = _lib.AdamHparams()
        # torch/optim/adam.py _multi_tensor_adam, capturable=False: python-float bias corrections
        bc1 = 1 - beta1 ** step
        bc2 = 1 - beta2 ** step
        h.neg_step_size = (lr / bc1) * -1
        h.one_minus_beta1 = 1 - beta1
        h.beta2 = beta2
        h.one_minus_beta2 = 1 - beta2
        h.bc2_sqrt = bc2 ** 0.5
        h.eps = group["eps"]
        h.decoupled = 1 if group["decoupled_weight_decay"] else 0
        h.weight_decay = wd if not h.decoupled else 0.0
        h.decay_mul = 1 - lr * wd if h.decoupled else 1.0
        return h

    def _launch(self, group, ps, gs, ms, vs, step, clip):
        L = _lib.lib()
        chunks = _Chunks.of([p.numel() for p in ps], ps[0].device)
        h = self._hparams(group, step)
        cp = _VP(clip.data_ptr()) if clip is not None else None
        s = _stream()
        for t0, t1, dev, n, _ in chunks.slices:
            _check(L.damc_adam_step(_VP(dev.data_ptr()), n, _ptrs(ps[t0:t1]), _ptrs(gs[t0:t1]), _ptrs(ms[t0:t1]),
                                    _ptrs(vs[t0:t1]), t1 - t0, ctypes.byref(h), cp, s), "damc_adam_step")

    def _run(self, clip=None, collected=None):
        for gi, group in enumerate(self.param_groups):
            ps, gs, ms, vs, steps = collected[gi] if collected is not None else self._collect(group)
            if not ps:
                continue
            common = self._advance_steps(group, steps)
            if common is not None:
                self._launch(group, ps, gs, ms, vs, common, clip)
                continue
            # parameters that joined the group at different steps: one launch per step value
            sv = torch.stack(steps)
            for val in sorted(set(sv.tolist())):
                idx = [i for i, x in enumerate(sv.tolist()) if x == val]
                self._launch(group, [ps[i] for i in idx], [gs[i] for i in idx], [ms[i] for i in idx],
                             [vs[i] for i in idx], val, clip)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._run()
        return loss

    @torch.no_grad()
    def clip_and_step(self, max_norm):
        """clip_grad_norm_(every parameter with a grad, max_norm) fused into the step; returns the total norm
        (0-d fp32 device tensor, as clip_grad_norm_ returns)."""
        collected = [self._collect(g) for g in self.param_groups]
        grads = [g for c in collected for g in c[1]]
        if not grads:
            return torch.tensor(0.0)
        out = _norm(_Chunks.of([g.numel() for g in grads], grads[0].device), grads, max_norm)
        self._run(clip=out, collected=collected)
        self.last_grad_norm = out[0]
        return out[0]


class AdamW(Adam):
    """torch.optim.AdamW (decoupled weight decay) on ``damc_adam_step``."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         foreach=foreach, maximize=maximize, capturable=capturable, differentiable=differentiable,
                         fused=fused, decoupled_weight_decay=True)


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False, foreach=None):
    """torch.nn.utils.clip_grad_norm_ (L2 only) on the HIP norm + scale kernels; returns the total norm."""
    if float(norm_type) != 2.0:
        raise NotImplementedError("damc.optim.clip_grad_norm_: norm_type 2 only")
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    for g in grads:
        _require_fp32_cuda(g, "grad")
    chunks = _Chunks.of([g.numel() for g in grads], grads[0].device)
    out = _norm(chunks, grads, max_norm)
    total = out[0]
    if error_if_nonfinite and bool(torch.logical_or(total.isnan(), total.isinf())):
        raise RuntimeError("The total norm of order 2.0 for gradients from `parameters` is non-finite")
    L = _lib.lib()
    s = _stream()
    for t0, t1, dev, n, _ in chunks.slices:
        _check(L.damc_grad_scale(_VP(dev.data_ptr()), n, _ptrs(grads[t0:t1]), t1 - t0, _VP(out.data_ptr()), s),
               "damc_grad_scale")
    return total
