"""Multi-GPU: one process per GPU (torchrun), chains sharded by GLOBAL index, RCCL only at the end.

The Langevin / reverse-sweep updates of different chains never interact (every term of U is a sum
over chains; InstanceNorm is per sample — SURVEY.md §8e), so a batch is split into contiguous
per-rank slices and each rank runs the HIP kernels on its slice with ``chain_base`` = the slice
start: Philox noise is keyed by the global chain index, so the union of the shards is bitwise the
1-GPU result.  The only collectives are the final reductions below (``all_reduce(SUM)`` over
RCCL/xGMI for backend "nccl", or gloo in the CPU tests):
  * reconstruction MSE (eval_gen_recon.py:177-212): [sum of per-sample MSE, count];
  * FID sufficient statistics (MCMC.py:130-176 feed pfw.fid): [sum f, sum f f^T, n] in fp64.
"""
import torch


def shard(global_batch, rank, world):
    """Contiguous balanced slice of [0, global_batch): returns (start, count)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world %d/%d" % (rank, world))
    base, rem = divmod(int(global_batch), int(world))
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def _dist():
    import torch.distributed as d

    return d if d.is_available() and d.is_initialized() else None


def all_reduce_sum_(t):
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t, op=d.ReduceOp.SUM)
    return t


class ReconMSE:
    """Running sum of per-sample mean squared reconstruction errors (eval_gen_recon.py:192-211)."""

    def __init__(self, device):
        self.acc = torch.zeros(2, dtype=torch.float64, device=device)

    def update(self, x_hat, x):
        per_sample = torch.mean((x_hat - x) ** 2, dim=list(range(1, x.dim())))
        self.acc[0] += per_sample.double().sum()
        self.acc[1] += per_sample.numel()

    def compute(self):
        tot = all_reduce_sum_(self.acc.clone())
        return float(tot[0] / tot[1])


class FidStats:
    """Sufficient statistics of feature vectors for the Frechet distance: sum f, sum f f^T, n (fp64).

    The feature extractor (Inception, third-party, unavailable offline) is outside the hot path;
    this class only shards and reduces its outputs, and the plain fp64 GEMM goes to the vendor BLAS.
    """

    def __init__(self, dim, device):
        self.s1 = torch.zeros(dim, dtype=torch.float64, device=device)
        self.s2 = torch.zeros(dim, dim, dtype=torch.float64, device=device)
        self.n = torch.zeros(1, dtype=torch.float64, device=device)

    def update(self, feats):
        f = feats.double().reshape(feats.shape[0], -1)
        self.s1 += f.sum(0)
        self.s2 += f.t() @ f
        self.n += f.shape[0]

    def compute(self):
        flat = torch.cat([self.s1, self.s2.reshape(-1), self.n])
        all_reduce_sum_(flat)
        d = self.s1.numel()
        s1, s2, n = flat[:d], flat[d:d + d * d].reshape(d, d), float(flat[-1])
        mu = s1 / n
        sigma = (s2 - n * torch.outer(mu, mu)) / (n - 1)
        return mu, sigma


def sharded_recon_mse(Q, G, E, batches, g_l_steps=10, g_llhd_sigma=0.1, g_l_step_size=0.1):
    """Eval reconstruction MSE over global batches, each split across ranks (eval_gen_recon.py:177-212).

    batches: iterable of global x batches (identical on every rank); rank r processes its slice.
    """
    from . import langevin

    d = _dist()
    rank, world = (d.get_rank(), d.get_world_size()) if d is not None else (0, 1)
    meter = None
    for x in batches:
        s, c = shard(x.shape[0], rank, world)
        if c == 0:
            continue
        xs = x[s:s + c].contiguous()
        meter = meter or ReconMSE(xs.device)
        with torch.no_grad():
            z = Q(xs)
        langevin.posterior_langevin(z, xs, G, E, g_l_steps, g_llhd_sigma, g_l_step_size, False, chain_base=s)
        meter.update(langevin.generator_forward(z, G), xs)
    if meter is None:
        meter = ReconMSE(torch.device("cuda"))
    return meter.compute()
