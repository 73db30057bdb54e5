"""Device plans: turn the reference's nn.Modules into packed descriptors for libdamc.

A plan reads the module structure once (layer kinds, shapes, activations) and, on every
call, re-packs the live parameters into device buffers it owns (the nets are trained
between Langevin calls, and EMA copies update through ``.data``, so nothing is cached
across calls except the buffers themselves).

Generator structure: ``_netG_*.gen`` = [ConvTranspose2d, LeakyReLU(.2)]* ConvTranspose2d, Tanh
(workspace/src/diffusion_net.py:20-203), or the toy MLP ``G.net`` = [Linear, ReLU]* Linear
(workspace/toy_example/toy_example.py:22-47).
EBM structure: ``_netE.ebm`` = Linear, LeakyReLU(.2), Linear, LeakyReLU(.2), Linear
(workspace/src/diffusion_net.py:207-223).
"""
import contextlib
import ctypes
import threading
import weakref

import torch

from . import _lib
from ._lib import check, ptr


def _act_of(mod):
    if isinstance(mod, torch.nn.LeakyReLU):
        return _lib.ACT_LRELU, float(mod.negative_slope)
    if isinstance(mod, torch.nn.ReLU):
        return _lib.ACT_LRELU, 0.0
    if isinstance(mod, torch.nn.Tanh):
        return _lib.ACT_TANH, 0.0
    raise NotImplementedError("unsupported activation %r" % (mod,))


def _sn_hook(m):
    from torch.nn.utils.spectral_norm import SpectralNorm

    for h in m._forward_pre_hooks.values():
        if isinstance(h, SpectralNorm):
            return h
    return None


def _require_plain_param(m):
    """A layer whose weight the plan can read: a plain parameter, or nn.utils.spectral_norm's (the reference's sn,
    diffusion_net.py:8-16) recomputed by _live_weight."""
    if hasattr(m, "weight_orig") and _sn_hook(m) is None:
        raise NotImplementedError("a reparametrised weight other than nn.utils.spectral_norm's")


_SN = threading.local()  # set while spectral_norm_step's power iteration is the one the current forward runs


def _live_weight(m):
    """The weight m's forward would use.  A spectral-norm layer (use_spc_norm=True generators, e_sn=True EBMs:
    diffusion_net.py:8-16, 21-44, 208-210) recomputes it in its forward pre-hook from weight_orig and the u, v vectors.
    In eval mode -- the mode the reference runs G and E in for the Langevin chains and the sweeps
    (train_gen_recon.py:191-193) -- without a power iteration, so the value is fixed and is what every forward of the
    chain would use: it is computed here the way the hook does and set as the hook sets it.  In train mode every
    forward advances u and v once: the caller runs that forward's power iteration first (spectral_norm_step), and the
    weight it set is the one read here."""
    h = _sn_hook(m)
    if h is None:
        return m.weight
    if m.training:
        if not getattr(_SN, "on", False):
            raise NotImplementedError("spectral-norm layer in train mode outside spectral_norm_step: its forward "
                                      "would run a power iteration")
        return getattr(m, h.name)
    with torch.no_grad():
        w = h.compute_weight(m, do_power_iteration=False)
    setattr(m, h.name, w)
    return w


def sn_train_layers(modules):
    """(module, SpectralNorm hook) of every layer in train mode with nn.utils.spectral_norm among modules."""
    out = []
    for m in modules:
        h = _sn_hook(m)
        if h is not None and m.training:
            out.append((m, h))
    return out


@contextlib.contextmanager
def spectral_norm_step(layers):
    """One reference forward's worth of nn.utils.spectral_norm in train mode (torch/nn/utils/spectral_norm.py,
    SpectralNorm.__call__ -> compute_weight(do_power_iteration=True)): each layer's u and v advance by the hook's own
    power iteration, in place, and the normalised weight is set on the module as the hook sets it; inside the block
    the plans pack that weight.  The reference's Langevin step calls netG(z) and netE(z) once each (MCMC.py:32,54-58),
    so a chain in train mode runs one of these per step, and u, v, the weights and z follow the reference's."""
    if layers:
        with torch.no_grad():
            for m, h in layers:
                setattr(m, h.name, h.compute_weight(m, do_power_iteration=True))
    prev = getattr(_SN, "on", False)
    _SN.on = True
    try:
        yield
    finally:
        _SN.on = prev


class GeneratorPlan:
    """Packed generator for damc_posterior_langevin / damc_generator_forward."""

    def __init__(self, G):
        seq = G.gen if hasattr(G, "gen") else G.net
        mods = list(seq)
        specs = []  # (module, act, slope)
        for m in mods:
            if isinstance(m, (torch.nn.ConvTranspose2d, torch.nn.Linear)):
                _require_plain_param(m)
                specs.append([m, _lib.ACT_NONE, 0.0])
            else:
                if not specs:
                    raise NotImplementedError("activation before the first layer")
                specs[-1][1], specs[-1][2] = _act_of(m)
        if not specs or len(specs) > _lib.MAX_LAYERS:
            raise NotImplementedError("generator with %d layers" % len(specs))
        self.modules = [s[0] for s in specs]
        first = self.modules[0]
        self.nz = first.in_channels if isinstance(first, torch.nn.ConvTranspose2d) else first.in_features
        layers = []
        h = 1
        for i, (m, act, slope) in enumerate(specs):
            last = i == len(specs) - 1
            L = dict(act=act, slope=slope)
            if isinstance(m, torch.nn.Linear):
                L.update(kind=_lib.LAYER_LINEAR, cin=m.in_features, cout=m.out_features, k=1, stride=1, pad=0,
                         hin=1, hout=1)
            else:
                k, s, p = m.kernel_size[0], m.stride[0], m.padding[0]
                if m.kernel_size[0] != m.kernel_size[1] or m.stride[0] != m.stride[1] or m.padding[0] != m.padding[1]:
                    raise NotImplementedError("non-square ConvTranspose2d")
                if m.output_padding != (0, 0) or m.dilation != (1, 1) or m.groups != 1:
                    raise NotImplementedError("ConvTranspose2d with output_padding/dilation/groups")
                hout = (h - 1) * s - 2 * p + k
                if i == 0:
                    kind = _lib.LAYER_PROJ
                elif last:
                    kind = _lib.LAYER_SMALLC
                else:
                    kind = _lib.LAYER_UP2
                L.update(kind=kind, cin=m.in_channels, cout=m.out_channels, k=k, stride=s, pad=p, hin=h, hout=hout)
                h = hout
            layers.append(L)
        self.layers = layers
        self.is_conv = layers[0]["kind"] != _lib.LAYER_LINEAR
        last = layers[-1]
        self.nc = last["cout"]
        self.h = self.w = last["hout"]
        self.device = None
        self.buffers = None
        self.desc = None

    # --------------------------------------------------------------------------------
    def _alloc(self, device):
        L = _lib.lib()
        self.device = device
        self.buffers = []
        desc = _lib.Generator()
        desc.n_layers = len(self.layers)
        desc.nz = self.nz
        desc.nc, desc.h, desc.w = self.nc, self.h, self.w
        for i, spec in enumerate(self.layers):
            d = desc.layers[i]
            d.kind = spec["kind"]
            d.cin, d.cout, d.k = spec["cin"], spec["cout"], spec["k"]
            d.stride, d.pad = spec["stride"], spec["pad"]
            d.hin = d.win = spec["hin"]
            d.hout = d.wout = spec["hout"]
            d.act, d.slope = spec["act"], spec["slope"]
            fwd, bwd = ctypes.c_size_t(), ctypes.c_size_t()
            check(L.damc_generator_layer_packed_sizes(ctypes.byref(d), ctypes.byref(fwd), ctypes.byref(bwd)),
                  "packed sizes")
            wf = torch.empty(max(int(fwd.value), 1), dtype=torch.float32, device=device)
            wb = torch.empty(max(int(bwd.value), 1), dtype=torch.float32, device=device)
            self.buffers.append((wf, wb))
            d.w_fwd = wf.data_ptr()
            d.w_bwd = wb.data_ptr() if bwd.value else None
        self.desc = desc

    def refresh(self, device, engine=None):
        """(Re)pack the live parameters; returns a per-call copy of the ctypes descriptor (so threads asking for
        different engines never share one).  engine: _lib.ENGINE_* for every layer (default:
        _lib.current_engine() of the calling thread)."""
        device = torch.device(device)
        engine = _lib.current_engine() if engine is None else int(engine)
        if device.type != "cuda":
            raise _lib.DamcError("the HIP generator path needs CUDA (ROCm) tensors, got %s" % device)
        if self.device != device or self.desc is None:
            self._alloc(device)
        L = _lib.lib()
        stream = _lib.stream_ptr(device)
        self._keep = []
        for i, m in enumerate(self.modules):
            w = _live_weight(m).detach()
            if w.device != device or w.dtype != torch.float32 or not w.is_contiguous():
                w = w.to(device=device, dtype=torch.float32).contiguous()
                self._keep.append(w)
            wf, wb = self.buffers[i]
            d = self.desc.layers[i]
            check(L.damc_pack_generator_layer(ctypes.byref(d), ptr(w), ptr(wf),
                                              ptr(wb) if d.w_bwd else None, stream), "pack generator layer")
            if m.bias is not None:
                b = m.bias.detach()
                if b.device != device or b.dtype != torch.float32:
                    b = b.to(device=device, dtype=torch.float32).contiguous()
                    self._keep.append(b)
                d.bias = b.data_ptr()
            else:
                d.bias = None
        out = _lib.Generator.from_buffer_copy(self.desc)
        for i in range(out.n_layers):
            out.layers[i].engine = engine
        return out

    def sn_train(self):
        return sn_train_layers(self.modules)

    def workspace(self, batch):
        L = _lib.lib()
        nbytes = int(L.damc_posterior_workspace_bytes(ctypes.byref(self.desc), int(batch)))
        if nbytes == 0:
            raise _lib.DamcError("unsupported generator configuration for the HIP path")
        if getattr(self, "_ws", None) is None:
            self._ws = _lib.WorkspaceCache()
        return self._ws.get(self.device, nbytes, int(batch)), nbytes


class EbmPlan:
    """_netE parameters + packed transposes."""

    def __init__(self, E):
        lin = [m for m in E.ebm if isinstance(m, torch.nn.Linear)]
        acts = [m for m in E.ebm if not isinstance(m, torch.nn.Linear)]
        if len(lin) != 3 or len(acts) != 2 or lin[2].out_features != 1:
            raise NotImplementedError("unexpected _netE structure")
        for m in lin:
            _require_plain_param(m)
        slopes = {float(a.negative_slope) for a in acts if isinstance(a, torch.nn.LeakyReLU)}
        if len(slopes) != 1:
            raise NotImplementedError("_netE activations must be LeakyReLU with one slope")
        self.slope = slopes.pop()
        self.lin = lin
        self.nz, self.nh = lin[0].in_features, lin[0].out_features
        self.device = None

    def sn_train(self):
        return sn_train_layers(self.lin)

    def refresh(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise _lib.DamcError("the HIP EBM path needs CUDA (ROCm) tensors, got %s" % device)
        self._keep = []

        def dev(t):
            t = t.detach()
            if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
                t = t.to(device=device, dtype=torch.float32).contiguous()
                self._keep.append(t)
            return t

        (w1, b1), (w2, b2), (w3, b3) = [(dev(_live_weight(m)), dev(m.bias)) for m in self.lin]
        if self.device != device:
            self.w1t = torch.empty(self.nz * self.nh, dtype=torch.float32, device=device)
            self.w2t = torch.empty(self.nh * self.nh, dtype=torch.float32, device=device)
            self.device = device
        d = _lib.Ebm()
        d.nz, d.nh, d.slope = self.nz, self.nh, self.slope
        d.w1, d.b1, d.w2, d.b2, d.w3, d.b3 = [t.data_ptr() for t in (w1, b1, w2, b2, w3, b3)]
        d.w1t, d.w2t = self.w1t.data_ptr(), self.w2t.data_ptr()
        self._params = (w1, b1, w2, b2, w3, b3)
        check(_lib.lib().damc_pack_ebm(ctypes.byref(d), ptr(self.w1t), ptr(self.w2t), _lib.stream_ptr(device)),
              "pack ebm")
        self.desc = d
        return d


_GEN_PLANS = weakref.WeakKeyDictionary()
_EBM_PLANS = weakref.WeakKeyDictionary()


def generator_plan(G):
    p = _GEN_PLANS.get(G)
    if p is None:
        p = GeneratorPlan(G)
        _GEN_PLANS[G] = p
    return p


def ebm_plan(E):
    p = _EBM_PLANS.get(E)
    if p is None:
        p = EbmPlan(E)
        _EBM_PLANS[E] = p
    return p
