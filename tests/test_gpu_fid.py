"""GPU: FID statistics on the HIP path (workspace/src/MCMC.py:130-176).

damc_fid_accumulate / damc_fid_mean_cov against np.mean / np.cov in fp64 on fixed feature arrays (streamed in
uneven chunks, as calculate_fid's batches arrive), and damc.fid.frechet_distance (pytorch-fid's algorithm)
against the oracle's independent eigenvalue form.  The Inception features themselves are third-party and
unavailable offline: FID values are parity unpinned; these tests pin everything downstream of the features.
Tolerances: statistics rel 1e-12 (fp64 sums of fp32 inputs in a different order), distance rel 1e-6 (sqrtm)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,chunks", [(1000, 64, (1, 499, 500)), (700, 2048, (300, 400)), (33, 130, (33,))])
def test_fid_statistics_match_numpy(gpu_device, n, d, chunks):
    from damc import fid
    from oracle import fid_oracle

    rng = np.random.default_rng(d)
    feats = (np.abs(rng.standard_normal((n, d))) * rng.uniform(0.1, 3.0, d)).astype(np.float32)
    acc = fid.FidAccumulator(d, gpu_device)
    o = 0
    for c in chunks:
        acc.update(torch.from_numpy(feats[o:o + c]).to(gpu_device))
        o += c
    assert acc.n == n
    mu, sigma = acc.compute()
    mu_ref, sigma_ref = fid_oracle.stats(feats)
    mu, sigma = mu.cpu().numpy(), sigma.cpu().numpy()
    assert np.abs(mu - mu_ref).max() <= 1e-12 * np.abs(mu_ref).max()
    assert np.abs(sigma - sigma_ref).max() <= 1e-11 * np.abs(sigma_ref).max()
    assert np.array_equal(sigma, sigma.T)


def test_frechet_distance_matches_oracle(gpu_device):
    from damc import fid
    from oracle import fid_oracle

    rng = np.random.default_rng(0)
    d = 256
    a = rng.standard_normal((2000, d)).astype(np.float32)
    b = (0.8 * rng.standard_normal((2000, d)) + 0.3).astype(np.float32)
    accs = []
    for f in (a, b):
        acc = fid.FidAccumulator(d, gpu_device)
        acc.update(torch.from_numpy(f).to(gpu_device))
        accs.append(acc.compute())
    (m1, s1), (m2, s2) = accs
    got = fid.frechet_distance(m1, s1, m2, s2)
    want = fid_oracle.frechet_distance(*fid_oracle.stats(a), *fid_oracle.stats(b))
    assert abs(got - want) <= 1e-6 * abs(want)
    assert abs(fid.frechet_distance(m1, s1, m1, s1)) < 1e-6 * np.trace(s1.cpu().numpy())


def test_fid_accumulator_refuses_cpu():
    from damc import _lib, fid

    with pytest.raises(_lib.DamcError):
        fid.FidAccumulator(8, "cpu")
