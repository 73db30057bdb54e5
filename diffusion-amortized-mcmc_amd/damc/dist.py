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


def block_plan(global_batch, rank, world, scaling="weak"):
    """Which chains one rank runs in a Langevin block (bench.py; train_gen_recon.py:203-209: posterior on B
    chains, prior on 2B = cat(z0, N(0, I)) chains), and the global index of its first chain of each kind.

    weak:   every rank runs a full batch of its own (B posterior + 2B prior chains); rank r's chains are
            global chains [r B, (r+1) B) and [2 r B, 2 (r+1) B) -> noise streams never collide.
    strong: the global batch is split: posterior rows shard(B) and prior rows shard(2B) of the global
            arrays; chain_base = the slice start, so the union over ranks is the 1-GPU block bit for bit.
    Returns dict(post_start, post_count, prior_start, prior_count, post_global, prior_global) — *_start are the
    chain_base values (and, for strong, the slice offsets into the global inputs); *_global the chain count of the
    block a rank's slice belongs to (what a shape-dependent engine choice must key on: langevin.prior_langevin's
    global_batch)."""
    B = int(global_batch)
    if scaling == "weak":
        return dict(post_start=rank * B, post_count=B, prior_start=rank * 2 * B, prior_count=2 * B,
                    post_global=B, prior_global=2 * B)
    if scaling == "strong":
        ps, pc = shard(B, rank, world)
        qs, qc = shard(2 * B, rank, world)
        return dict(post_start=ps, post_count=pc, prior_start=qs, prior_count=qc, post_global=B, prior_global=2 * B)
    raise ValueError("scaling must be 'weak' or 'strong', got %r" % (scaling,))


def _dist():
    import torch.distributed as d

    return d if d.is_available() and d.is_initialized() else None


def all_reduce_sum_(t, group=None):
    d = _dist()
    if d is not None and d.get_world_size(group) > 1:
        d.all_reduce(t, op=d.ReduceOp.SUM, group=group)
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
    Every rank draws the same global initial latents and sweep key from its (identically seeded) torch
    generator and runs its slice with chain_base = the slice start, so the Q sweep and the posterior
    chains of the union of the shards are bitwise the 1-GPU run's.
    """
    from . import amortizer, langevin

    d = _dist()
    rank, world = (d.get_rank(), d.get_world_size()) if d is not None else (0, 1)
    meter = None
    for x in batches:
        s, c = shard(x.shape[0], rank, world)
        # global draws, identical on every rank (host generator), in q_forward's order: zt, then the sweep key
        zt = torch.randn(x.shape[0], Q.nz)
        seed = langevin.new_seed() if Q.with_noise else 0
        if c == 0:
            continue
        xs = x[s:s + c].contiguous()
        meter = meter or ReconMSE(xs.device)
        with torch.no_grad():
            z = amortizer.q_forward(Q, x=xs, zt=zt[s:s + c], seed=seed, chain_base=s)
        langevin.posterior_langevin(z, xs, G, E, g_l_steps, g_llhd_sigma, g_l_step_size, False, chain_base=s)
        meter.update(langevin.generator_forward(z, G), xs)
    if meter is None:
        meter = ReconMSE(torch.device("cuda"))
    return meter.compute()
