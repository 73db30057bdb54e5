"""TEST INFRASTRUCTURE ONLY (never imported by the product path): FID statistics and distance as the reference
computes them.

workspace/src/MCMC.py:130-176 calls pytorch_fid_wrapper 0.0.4's ``pfw.fid(images, real_m, real_s)``, which
(third-party, unvendored; README.md:16-17 pins pytorch-fid 0.2.1 / pytorch-fid-wrapper 0.0.4) reduces the
Inception pool features with ``np.mean(act, axis=0)`` / ``np.cov(act, rowvar=False)`` and returns pytorch-fid's
``calculate_frechet_distance``: |mu1 - mu2|^2 + tr(S1) + tr(S2) - 2 tr(sqrtm(S1 S2)).  Restated here in fp64
numpy with an independent trace term: for PSD S1, S2 the eigenvalues of S1 S2 are those of the symmetric
S1^1/2 S2 S1^1/2, so tr sqrtm(S1 S2) = sum sqrt(eigvalsh(S1^1/2 S2 S1^1/2)) (no Schur-form sqrtm)."""
import numpy as np


def stats(feats):
    f = np.asarray(feats, dtype=np.float64)
    return f.mean(axis=0), np.cov(f, rowvar=False)


def _psd_sqrt(s):
    w, v = np.linalg.eigh(s)
    return (v * np.sqrt(np.clip(w, 0.0, None))) @ v.T


def frechet_distance(mu1, s1, mu2, s2):
    mu1, mu2, s1, s2 = (np.asarray(a, dtype=np.float64) for a in (mu1, mu2, s1, s2))
    r = _psd_sqrt(s1)
    tr_covmean = np.sum(np.sqrt(np.clip(np.linalg.eigvalsh(r @ s2 @ r), 0.0, None)))
    d = mu1 - mu2
    return float(d @ d + np.trace(s1) + np.trace(s2) - 2.0 * tr_covmean)
