"""FID on the HIP path: device-side sufficient statistics, one RCCL all_reduce, then the
Frechet distance of pytorch-fid 0.2.1 (the algorithm pytorch_fid_wrapper's ``pfw.fid`` applies in
workspace/src/MCMC.py:130-176).

  acc = FidAccumulator(dim, device); acc.update(features) per batch  -> damc_fid_accumulate (fp64 s1, s2)
  mu, sigma = acc.compute()                                        -> this rank's samples, damc_fid_mean_cov
  mu, sigma = acc.compute(reduce=True, group=g)                    -> sharded FID: all_reduce(SUM) of s1, s2, n
                                                                      over the group first (RCCL for "nccl")
  fid = frechet_distance(mu, sigma, real_m, real_s)                -> host fp64 (scipy.linalg.sqrtm), exactly
                                                                      pytorch-fid's calculate_frechet_distance

The Inception-v3 feature extractor is third-party (pytorch-fid's pretrained weights, unavailable offline), so
FID values themselves are "parity unpinned"; the statistics and the distance are pinned against numpy / scipy
in tests/test_gpu_fid.py.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr


class FidAccumulator:
    """Running fp64 (sum f, sum f f^T, n) of feature rows on one GPU."""

    def __init__(self, dim, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise _lib.DamcError("FidAccumulator runs on a ROCm device (the HIP path has no CPU fallback)")
        self.dim, self.device = int(dim), device
        self.s1 = torch.zeros(self.dim, dtype=torch.float64, device=device)
        self.s2 = torch.zeros(self.dim, self.dim, dtype=torch.float64, device=device)
        self.n = 0

    def update(self, feats):
        f = feats.detach().reshape(feats.shape[0], -1)
        if f.shape[1] != self.dim:
            raise _lib.DamcError("features of width %d for a %d-wide accumulator" % (f.shape[1], self.dim))
        f = f.to(device=self.device, dtype=torch.float32).contiguous()
        check(_lib.lib().damc_fid_accumulate(ptr(f), f.shape[0], self.dim, ptr(self.s1), ptr(self.s2),
                                             _lib.stream_ptr(self.device)), "damc_fid_accumulate")
        self.n += f.shape[0]

    def compute(self, reduce=False, group=None):
        """(mu, sigma) as fp64 device tensors.

        reduce=False (default): this accumulator's samples only, like the reference's single ``pfw.fid`` call; no
        collective, so a driver that computes FID on rank 0 alone cannot deadlock.  reduce=True: the sharded FID,
        every rank of ``group`` (default: the world) calls compute(reduce=True) and gets the statistics of the
        union of their samples (one all_reduce of s1, s2 and n; each rank's tensors stay on its own device)."""
        flat = torch.cat([self.s1, self.s2.reshape(-1),
                          torch.tensor([float(self.n)], dtype=torch.float64, device=self.device)])
        if reduce:
            from .dist import all_reduce_sum_

            all_reduce_sum_(flat, group=group)
        d = self.dim
        s1, s2, n = flat[:d].contiguous(), flat[d:d + d * d].contiguous(), float(flat[-1].item())
        mu = torch.empty(d, dtype=torch.float64, device=self.device)
        sigma = torch.empty(d, d, dtype=torch.float64, device=self.device)
        check(_lib.lib().damc_fid_mean_cov(ptr(s1), ptr(s2), n, d, ptr(mu), ptr(sigma),
                                           _lib.stream_ptr(self.device)), "damc_fid_mean_cov")
        return mu, sigma


def frechet_distance(mu1, sigma1, mu2, sigma2, eps=1e-6):
    """pytorch-fid 0.2.1 calculate_frechet_distance (fp64 numpy / scipy.linalg.sqrtm), the reference's FID."""
    from scipy import linalg

    mu1, mu2 = np.atleast_1d(_np(mu1)), np.atleast_1d(_np(mu2))
    sigma1, sigma2 = np.atleast_2d(_np(sigma1)), np.atleast_2d(_np(sigma2))
    if mu1.shape != mu2.shape or sigma1.shape != sigma2.shape:
        raise ValueError("mean vectors / covariances of different shapes")
    diff = mu1 - mu2
    covmean, _ = linalg.sqrtm(sigma1.dot(sigma2), disp=False)
    if not np.isfinite(covmean).all():
        offset = np.eye(sigma1.shape[0]) * eps
        covmean = linalg.sqrtm((sigma1 + offset).dot(sigma2 + offset))
    if np.iscomplexobj(covmean):
        if not np.allclose(np.diagonal(covmean).imag, 0, atol=1e-3):
            raise ValueError("imaginary component %g" % np.max(np.abs(covmean.imag)))
        covmean = covmean.real
    return float(diff.dot(diff) + np.trace(sigma1) + np.trace(sigma2) - 2 * np.trace(covmean))


def _np(a):
    return a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, dtype=np.float64)


def inception_features(images, batch_size=200):
    """pool3 features of images in [0, 1] (N, 3, H, W) with pytorch-fid's InceptionV3 (third-party; its weights
    are downloaded by that package, so this is unavailable offline and raises ImportError here)."""
    from pytorch_fid.inception import InceptionV3  # noqa: F401  third-party, not vendored

    dev = images.device
    model = InceptionV3([InceptionV3.BLOCK_INDEX_BY_DIM[2048]]).to(dev).eval()
    out = []
    with torch.no_grad():
        for i in range(0, images.shape[0], batch_size):
            out.append(model(images[i:i + batch_size])[0].reshape(-1, 2048))
    return torch.cat(out)


def fid_of_samples(samples, real_m, real_s, device=None):
    """pfw.fid(samples, real_m, real_s) on the HIP statistics path: features -> accumulate -> Frechet."""
    feats = inception_features(samples)
    acc = FidAccumulator(feats.shape[1], device or feats.device)
    acc.update(feats)
    mu, sigma = acc.compute()
    return frechet_distance(mu, sigma, real_m, real_s)
