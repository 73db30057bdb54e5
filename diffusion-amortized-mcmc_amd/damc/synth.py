"""Counter-hash synthetic data: weights, images, latents and injected noise.

Every tensor the parity tests and the bench use is a pure function of
``(seed, stream, element index)`` through splitmix64, so the golden-fixture
script (run once in the build container against the reference) and the tests
(run anywhere, including the GPU box where the reference does not exist)
regenerate bit-identical inputs without any torch RNG dependency.

Recipe (SURVEY.md §8c "Golden-vector recipe"):
  * uniform(seed, stream, n)  -> float64 in [0, 1) from the top 53 bits
  * normal(seed, stream, n)   -> Box-Muller over two uniform streams
  * weights: parameter #t of ``state_dict`` order gets stream t and is drawn
    U[-b, b] with b = 1/sqrt(fan_in), fan_in = shape[1] * prod(shape[2:])
    (the same bound rule torch's default Linear/Conv init uses); 1-D params
    take the bound of the preceding weight.  InstanceNorm affine weights are
    1 + 0.1 u, their biases 0.1 u; ``p.B`` and ``xemb`` are N(0, 1), matching
    the reference's ``torch.randn`` parameters
    (workspace/src/diffusion_net.py:479,576).
"""
import math

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def _mix(x):
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += _GOLDEN
        x = (x ^ (x >> np.uint64(30))) * _C1
        x = (x ^ (x >> np.uint64(27))) * _C2
        x = x ^ (x >> np.uint64(31))
    return x


def _key(seed, stream):
    s = np.array([seed & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64)
    t = np.array([stream & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix(_mix(s) ^ (t * _C1))[0]


def uniform(seed, stream, n):
    """n float64 values in [0, 1)."""
    idx = np.arange(n, dtype=np.uint64)
    bits = _mix(idx ^ _key(seed, stream))
    return (bits >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed, stream, n):
    """n float64 standard normals (Box-Muller, cos branch)."""
    u1 = uniform(seed, 2 * stream + 1, n)
    u2 = uniform(seed, 2 * stream + 2, n)
    r = np.sqrt(-2.0 * np.log(1.0 - u1))
    return r * np.cos(2.0 * math.pi * u2)


def uniform_f32(seed, stream, shape, lo=-1.0, hi=1.0):
    n = int(np.prod(shape))
    return (lo + (hi - lo) * uniform(seed, stream, n)).astype(np.float32).reshape(shape)


def normal_f32(seed, stream, shape):
    n = int(np.prod(shape))
    return normal(seed, stream, n).astype(np.float32).reshape(shape)


def _fan_in(shape):
    if len(shape) < 2:
        return None
    rf = 1
    for d in shape[2:]:
        rf *= int(d)
    return int(shape[1]) * rf


def state_dict_arrays(named_shapes, seed=0, norm_keys=(), normal_keys=("p.B", "xemb")):
    """Deterministic parameters for an ordered list of (name, shape).

    ``norm_keys``: names of InstanceNorm affine parameters (drawn near 1 / 0).
    Returns an ordered list of (name, float32 ndarray).
    """
    out = []
    last_bound = 1.0
    for t, (name, shape) in enumerate(named_shapes):
        shape = tuple(int(s) for s in shape)
        if name in normal_keys:
            arr = normal_f32(seed, 1000 + t, shape)
        elif name in norm_keys:
            u = uniform_f32(seed, 1000 + t, shape)
            arr = (1.0 + 0.1 * u) if name.endswith("weight") else 0.1 * u
            arr = arr.astype(np.float32)
        else:
            fi = _fan_in(shape)
            bound = last_bound if fi is None else 1.0 / math.sqrt(fi)
            if fi is not None:
                last_bound = bound
            arr = uniform_f32(seed, 1000 + t, shape, -bound, bound)
        out.append((name, arr))
    return out


def load_into(module, seed=0):
    """Fill an nn.Module's parameters/buffers in state_dict order (in place)."""
    import torch

    sd = module.state_dict()
    norm_keys = set()
    for mname, m in module.named_modules():
        if isinstance(m, torch.nn.InstanceNorm2d):
            norm_keys.add(mname + ".weight")
            norm_keys.add(mname + ".bias")
    shapes = [(k, tuple(v.shape)) for k, v in sd.items() if v.dtype.is_floating_point]
    arrays = dict(state_dict_arrays(shapes, seed=seed, norm_keys=norm_keys))
    new_sd = {}
    for k, v in sd.items():
        new_sd[k] = torch.from_numpy(arrays[k]).to(v.device) if k in arrays else v
    module.load_state_dict(new_sd)
    return module
