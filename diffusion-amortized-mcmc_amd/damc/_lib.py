"""ctypes binding of libdamc.so (include/damc.h).

The library is built in-tree (``make -C diffusion-amortized-mcmc_amd/csrc``) and loaded from
this directory.  There is deliberately NO fallback: if the .so is missing or a call fails,
``lib()`` / ``check()`` raise, so a GPU box never silently runs anything but the HIP path.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DAMC_LIB_PATH: an alternative in-tree build for A/B timing (tools/); the default is the product library
LIB_PATH = os.environ.get("DAMC_LIB_PATH") or os.path.join(_HERE, "libdamc.so")

ABI_VERSION = 3
MAX_LAYERS = 10
ENGINE_LIMB, ENGINE_FP32 = 0, 1
# include/damc.h error codes
DAMC_ERR_ARG, DAMC_ERR_WORKSPACE, DAMC_ERR_UNSUPPORTED = 1001, 1002, 1003
LAYER_PROJ, LAYER_UP2, LAYER_SMALLC, LAYER_LINEAR = 1, 2, 3, 4
ACT_NONE, ACT_LRELU, ACT_TANH = 0, 1, 2

c_float_p = ctypes.POINTER(ctypes.c_float)


class Layer(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int),
        ("cin", ctypes.c_int), ("cout", ctypes.c_int), ("k", ctypes.c_int),
        ("stride", ctypes.c_int), ("pad", ctypes.c_int),
        ("hin", ctypes.c_int), ("win", ctypes.c_int), ("hout", ctypes.c_int), ("wout", ctypes.c_int),
        ("act", ctypes.c_int), ("slope", ctypes.c_float),
        ("w_fwd", ctypes.c_void_p), ("w_bwd", ctypes.c_void_p), ("bias", ctypes.c_void_p),
        ("engine", ctypes.c_int),
    ]


class Generator(ctypes.Structure):
    _fields_ = [
        ("n_layers", ctypes.c_int), ("nz", ctypes.c_int),
        ("nc", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
        ("layers", Layer * MAX_LAYERS),
    ]


class GeneratorGrads(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p * MAX_LAYERS), ("b", ctypes.c_void_p * MAX_LAYERS)]


class Ebm(ctypes.Structure):
    _fields_ = [
        ("nz", ctypes.c_int), ("nh", ctypes.c_int), ("slope", ctypes.c_float),
        ("w1", ctypes.c_void_p), ("b1", ctypes.c_void_p), ("w2", ctypes.c_void_p),
        ("b2", ctypes.c_void_p), ("w3", ctypes.c_void_p), ("b3", ctypes.c_void_p),
        ("w1t", ctypes.c_void_p), ("w2t", ctypes.c_void_p),
    ]


class CsqBlock(ctypes.Structure):  # damc_csq_block_t
    _fields_ = [
        ("din", ctypes.c_int), ("dout", ctypes.c_int),
        ("wl", ctypes.c_void_p), ("bl", ctypes.c_void_p), ("ws", ctypes.c_void_p), ("bs", ctypes.c_void_p),
        ("wg", ctypes.c_void_p), ("bg", ctypes.c_void_p), ("wb", ctypes.c_void_p),
    ]


class Denoiser(ctypes.Structure):  # damc_denoiser_t (= damc_denoiser_train_t): PyTorch layouts throughout
    _fields_ = [
        ("nz", ctypes.c_int), ("ntemb", ctypes.c_int), ("nxemb", ctypes.c_int), ("residual", ctypes.c_int),
        ("bmat", ctypes.c_void_p),
        ("tw1", ctypes.c_void_p), ("tb1", ctypes.c_void_p), ("tw2", ctypes.c_void_p), ("tb2", ctypes.c_void_p),
        ("blocks", CsqBlock * 7),
        ("wctx", ctypes.c_void_p * 7), ("bctx", ctypes.c_void_p * 7),
    ]


DenoiserTrain = Denoiser


class DenoiserGrads(ctypes.Structure):
    _fields_ = [("bmat", ctypes.c_void_p), ("tw1", ctypes.c_void_p), ("tb1", ctypes.c_void_p),
                ("tw2", ctypes.c_void_p), ("tb2", ctypes.c_void_p)] + [
        (k, ctypes.c_void_p * 7) for k in ("wl", "bl", "ws", "bs", "wg", "bg", "wb", "wctx", "bctx")]


MAX_ENC_LAYERS = 8


class EncLayer(ctypes.Structure):  # damc_enc_layer_t
    _fields_ = [("cin", ctypes.c_int), ("cout", ctypes.c_int), ("k", ctypes.c_int), ("stride", ctypes.c_int),
                ("pad", ctypes.c_int), ("w_packed", ctypes.c_void_p), ("bias", ctypes.c_void_p),
                ("in_gamma", ctypes.c_void_p), ("in_beta", ctypes.c_void_p), ("in_eps", ctypes.c_float),
                ("slope", ctypes.c_float), ("w_x3", ctypes.c_void_p), ("w_src", ctypes.c_void_p)]


class Encoder(ctypes.Structure):  # damc_encoder_t
    _fields_ = [("n_layers", ctypes.c_int), ("nc", ctypes.c_int), ("h", ctypes.c_int), ("w", ctypes.c_int),
                ("layers", EncLayer * MAX_ENC_LAYERS), ("engine", ctypes.c_int)]


class EncoderGrads(ctypes.Structure):  # damc_encoder_grads_t
    _fields_ = [(k, ctypes.c_void_p * MAX_ENC_LAYERS) for k in ("w", "b", "gamma", "beta")]


class EbmGrads(ctypes.Structure):  # damc_ebm_grads_t
    _fields_ = [(k, ctypes.c_void_p) for k in ("w1", "b1", "w2", "b2", "w3", "b3")]


class PriorEmb(ctypes.Structure):  # damc_prior_emb_t
    _fields_ = [("nz", ctypes.c_int), ("nh", ctypes.c_int), ("nout", ctypes.c_int), ("slope", ctypes.c_float)] + [
        (k, ctypes.c_void_p) for k in ("w1", "b1", "w2", "b2")]


class PriorEmbGrads(ctypes.Structure):  # damc_prior_emb_grads_t
    _fields_ = [(k, ctypes.c_void_p) for k in ("w1", "b1", "w2", "b2")]


class AdamHparams(ctypes.Structure):
    _fields_ = [("neg_step_size", ctypes.c_float), ("one_minus_beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("one_minus_beta2", ctypes.c_float), ("bc2_sqrt", ctypes.c_float), ("eps", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("decay_mul", ctypes.c_float), ("decoupled", ctypes.c_int)]


ADAM_CHUNK = 8192
ADAM_MAX_TENSORS = 96


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_D = ctypes.c_double
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t

_SIGS = {
    "damc_abi_version": (_I, []),
    "damc_error_string": (ctypes.c_char_p, [_I]),
    "damc_generator_layer_packed_sizes": (_I, [ctypes.POINTER(Layer), ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    "damc_pack_generator_layer": (_I, [ctypes.POINTER(Layer), _P, _P, _P, _P]),
    "damc_pack_ebm": (_I, [ctypes.POINTER(Ebm), _P, _P, _P]),
    "damc_posterior_workspace_bytes": (_SZ, [ctypes.POINTER(Generator), _I]),
    "damc_posterior_langevin": (_I, [ctypes.POINTER(Generator), ctypes.POINTER(Ebm), _P, _P, _I, _I, _D, _D, _I, _P,
                                     _U64, _U64, _U64, _P, _P, _SZ, _P]),
    "damc_likelihood_grad": (_I, [ctypes.POINTER(Generator), _P, _P, _I, _D, _P, _P, _SZ, _P]),
    "damc_generator_forward": (_I, [ctypes.POINTER(Generator), _P, _I, _P, _P, _SZ, _P]),
    "damc_convT_workspace_bytes": (_SZ, [ctypes.POINTER(Layer), _I]),
    "damc_convT_fwd": (_I, [ctypes.POINTER(Layer), _P, _I, _P, _P, _SZ, _P]),
    "damc_convT_dgrad": (_I, [ctypes.POINTER(Layer), _P, _I, _P, _I, _F, _P, _P, _SZ, _P]),
    "damc_generator_train_workspace_bytes": (_SZ, [ctypes.POINTER(Generator), _I]),
    "damc_generator_train_forward": (_I, [ctypes.POINTER(Generator), _P, _I, _P, _P, _SZ, _P]),
    "damc_generator_train_backward": (_I, [ctypes.POINTER(Generator), _P, _P, _P, _I, ctypes.POINTER(GeneratorGrads),
                                           _P, _P, _SZ, _P]),
    "damc_denoiser_train_workspace_bytes": (_SZ, [ctypes.POINTER(DenoiserTrain), _I]),
    "damc_denoiser_train_forward": (_I, [ctypes.POINTER(DenoiserTrain), _P, _P, _P, _I, _P, _P, _SZ, _P]),
    "damc_denoiser_train_backward": (_I, [ctypes.POINTER(DenoiserTrain), _P, _I, ctypes.POINTER(DenoiserGrads), _P,
                                          _P, _P, _SZ, _P]),
    "damc_encoder_train_saved_floats": (_SZ, [ctypes.POINTER(Encoder), _I]),
    "damc_encoder_train_workspace_bytes": (_SZ, [ctypes.POINTER(Encoder), _I]),
    "damc_encoder_train_forward": (_I, [ctypes.POINTER(Encoder), _P, _I, _P, _P, _P, _SZ, _P]),
    "damc_encoder_train_backward": (_I, [ctypes.POINTER(Encoder), _P, _P, _I, ctypes.POINTER(EncoderGrads), _P, _SZ,
                                         _P]),
    "damc_ebm_train_workspace_bytes": (_SZ, [ctypes.POINTER(Ebm), _I]),
    "damc_ebm_train_forward": (_I, [ctypes.POINTER(Ebm), _P, _I, _P, _P, _P, _P]),
    "damc_ebm_train_backward": (_I, [ctypes.POINTER(Ebm), _P, _P, _P, _P, ctypes.c_long, _I, ctypes.POINTER(EbmGrads),
                                     _P, _P, _SZ, _P]),
    "damc_prior_emb_train_workspace_bytes": (_SZ, [ctypes.POINTER(PriorEmb), _I]),
    "damc_prior_emb_train_forward": (_I, [ctypes.POINTER(PriorEmb), _P, _I, _P, _P, _P]),
    "damc_prior_emb_train_backward": (_I, [ctypes.POINTER(PriorEmb), _P, _P, _P, _I, ctypes.POINTER(PriorEmbGrads), _P,
                                           _SZ, _P]),
    "damc_q_noise_glue": (_I, [_P, _P, _P, _I, _I, _F, _F, _P, _I, _P, _P, _P, _P]),
    "damc_q_loss_forward": (_I, [_P, _P, _I, _I, _P, _P]),
    "damc_q_loss_backward": (_I, [_P, _P, _P, ctypes.c_long, _I, _I, _P, _P]),
    "damc_prior_langevin": (_I, [ctypes.POINTER(Ebm), _P, _I, _I, _D, _I, _P, _U64, _U64, _U64, _P, _P]),
    "damc_prior_langevin_engine": (_I, [ctypes.POINTER(Ebm), _P, _I, _I, _D, _I, _P, _U64, _U64, _U64, _P, _I, _P]),
    "damc_ebm_mfma_min_chains": (_I, []),
    "damc_ebm_energy_grad": (_I, [ctypes.POINTER(Ebm), _P, _I, _P, _P, _P]),
    "damc_z_update": (_I, [_P, _P, _I, _I, _D, _I, _P, _U64, _U64, _U64, _P]),
    "damc_philox_normal": (_I, [_P, _I, _I, _I, _U64, _U64, _U64, ctypes.c_uint32, _P]),
    "damc_conv2d_workspace_floats": (_SZ, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "damc_conv2d_nhwc": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "damc_pack_conv2d": (_I, [_P, _I, _I, _I, _P, _P]),
    "damc_instnorm_workspace_floats": (_SZ, [_I, _I, _I]),
    "damc_instnorm_lrelu_train_nhwc": (_I, [_P, _I, _I, _I, _P, _P, _F, _F, _P, _P, _P, _P]),
    "damc_instnorm_bwd_workspace_floats": (_SZ, [_I, _I, _I]),
    "damc_instnorm_lrelu_backward_nhwc": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _F, _P, _P, _P, _P, _P]),
    "damc_conv2d_backward_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "damc_conv2d_backward_nhwc": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _SZ, _P]),
    "damc_instnorm_lrelu_nhwc": (_I, [_P, _I, _I, _I, _P, _P, _F, _F, _P, _P]),
    "damc_nchw_to_nhwc": (_I, [_P, _I, _I, _I, _P, _P]),
    "damc_q_encoder_workspace_bytes": (_SZ, [ctypes.POINTER(Encoder), _I]),
    "damc_q_encoder_fwd": (_I, [ctypes.POINTER(Encoder), _P, _I, _P, _P, _SZ, _P]),
    "damc_gemm": (_I, [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _I, _F, _P]),
    "damc_conv2d_x3_bytes": (_SZ, [_I, _I, _I]),
    "damc_x3_sign_block": (_I, []),
    "damc_x3_layer_sign_block": (_I, [ctypes.POINTER(Layer), _I]),
    "damc_conv2d_x3_workspace_bytes": (_SZ, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "damc_conv2d_x3_nhwc": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _P, _P, _SZ, _P]),
    "damc_clock_probe": (_I, [_P, _I]),
    "damc_x3_fixup_probe": (_I, [_P]),
    "damc_x3_conv_walk": (_I, [_I, _I]),
    "damc_pack_conv2d_x3": (_I, [_P, _I, _I, _I, _P, _P]),
    "damc_sweep_workspace_bytes": (_SZ, [ctypes.POINTER(Denoiser), _I, _I]),
    "damc_sweep_team_failures": (ctypes.c_long, [_I]),
    "damc_sweep_team_words": (_I, [ctypes.POINTER(Denoiser), _I, _I, _P, _SZ, _P, _I]),
    "damc_reverse_sweep": (_I, [ctypes.POINTER(Denoiser), _P, _P, _I, _I, _P, _P, _I, _P, _U64, _U64, _P, _I, _P,
                                _SZ, _P]),
    "damc_q_reverse_sweep": (_I, [ctypes.POINTER(Denoiser), _P, _P, _I, _I, _P, _P, _I, _P, _U64, _U64, _P, _I, _P,
                                  _SZ, _P]),
    "damc_denoise_step": (_I, [ctypes.POINTER(Denoiser), _P, _P, _I, _P, _P, _I, _P, _U64, _U64, _U64, _P, _P, _SZ,
                               _P]),
    "damc_ebm_grad": (_I, [ctypes.POINTER(Ebm), _P, _I, _P, _P, _P]),
    "damc_adam_chunk_bytes": (_SZ, []),
    "damc_adam_chunk_count": (_I, [ctypes.POINTER(ctypes.c_longlong), _I]),
    "damc_adam_build_chunks": (_I, [ctypes.POINTER(ctypes.c_longlong), _I, _P, _I]),
    "damc_grad_norm": (_I, [_P, _I, _P, _I, _F, _P, _P, _P]),
    "damc_grad_sumsq": (_I, [_P, _I, _P, _I, _P, _P]),
    "damc_grad_norm_finish": (_I, [_P, _I, _F, _P, _P]),
    "damc_grad_scale": (_I, [_P, _I, _P, _I, _P, _P]),
    "damc_adam_step": (_I, [_P, _I, _P, _P, _P, _P, _I, ctypes.POINTER(AdamHparams), _P, _P]),
    "damc_fid_accumulate": (_I, [_P, _I, _I, _P, _P, _P]),
    "damc_fid_mean_cov": (_I, [_P, _P, ctypes.c_double, _I, _P, _P, _P]),
    "damc_prof_enable": (_I, [_I]),
    "damc_prof_reset": (_I, []),
    "damc_prof_select": (_I, [ctypes.c_char_p]),
    "damc_prof_query": (_I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long),
                             ctypes.POINTER(ctypes.c_double)]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


class DamcError(RuntimeError):
    pass


def lib():
    """Load libdamc.so (raises if it was not built — there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DamcError(
                "libdamc.so not found at %s: build it with `make -C diffusion-amortized-mcmc_amd/csrc` "
                "(or __graft_entry__.build()); the HIP path has no fallback" % LIB_PATH)
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.damc_abi_version() != ABI_VERSION:
            raise DamcError("libdamc ABI mismatch")
        _lib = handle
    return _lib


_engine_state = threading.local()


def current_engine():
    """The generator convolution engine descriptors get when they are (re)packed on this thread:
    ENGINE_LIMB unless inside ``exact_fp32()`` (or DAMC_EXACT_FP32=1 in the environment)."""
    e = getattr(_engine_state, "engine", None)
    if e is None:
        e = ENGINE_FP32 if os.environ.get("DAMC_EXACT_FP32", "0") == "1" else ENGINE_LIMB
    return e


class exact_fp32:
    """Context manager: generator convolutions packed inside it run on the fp32-MFMA engine instead of the
    limb engine.  The choice is per thread and travels in each call's descriptor (no library-global state)."""

    def __init__(self, on=True):
        self.on = on

    def __enter__(self):
        self.prev = getattr(_engine_state, "engine", None)
        _engine_state.engine = ENGINE_FP32 if self.on else ENGINE_LIMB
        return self

    def __exit__(self, *exc):
        _engine_state.engine = self.prev
        return False


def check(rc, what=""):
    if rc != 0:
        msg = lib().damc_error_string(rc).decode()
        raise DamcError("%s failed: %s (code %d)" % (what or "damc call", msg, rc))
    return rc


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class WorkspaceCache:
    """A reusable device workspace per (thread, stream, key).  A library call's kernels are enqueued in order on
    the caller's stream, so two calls may share scratch memory only if they are ordered on the same stream and
    issued by the same thread: two threads on one stream interleave their launches (one call's kernels would
    overwrite the other's intermediates), and two streams run concurrently."""

    def __init__(self):
        self._tls = threading.local()

    def get(self, device, nbytes, key):
        import torch

        stream = torch.cuda.current_stream(device).cuda_stream
        k = (key, str(device), stream)
        cur = getattr(self._tls, "ws", None)
        if cur is None or cur[0] != k or cur[1].numel() < nbytes:
            self._tls.ws = cur = (k, torch.empty(nbytes, dtype=torch.uint8, device=device))
        return cur[1]
