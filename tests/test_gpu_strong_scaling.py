"""8-way strong scaling pinned at the per-rank kernels, on one MI355X.

The BASELINE multi-GPU configs split one global batch over 8 ranks (damc.dist.block_plan: contiguous slices,
chain_base = the slice start, Philox noise keyed by the global chain index; reference drivers
workspace/train_gen_recon.py:203-209, workspace/src/MCMC.py:27-74, workspace/src/diffusion_net.py:585-622).  A rank's
batch takes different kernels than the whole batch does -- the skinny first layer at <= 32 rows, km_skinny, split-K at
16 rows per tile (with its in-GEMM ordered fix-up), the direct gather, the sweep's team partition -- so each check
below runs the whole batch in one call and its 8 slices as 8 calls, and requires the concatenation of the slices to be
BITWISE the whole batch, over the full multi-step chains:

  * CIFAR-10 (headline): B=128, 30 noisy posterior steps, then 60 noisy prior steps on 2B=256 = 8 x (16, 32);
  * CelebA-64 (config 4): B=256, nz=100, 10 noisy posterior steps + 20 prior steps on 2B = 8 x (32, 64);
  * CelebA-HQ Q(x) (config 5): encoder + 100-step 'large' reverse sweep at B=64 = 8 x B=8;
  * bench.py --gpus 8 itself: 8 ranks sharing the GPU over gloo, the union of their chains = the 1-rank block.
"""
import numpy as np
import pytest
import torch

from test_gpu_dist import _run

pytestmark = pytest.mark.gpu

WORLD = 8


def _gen_case(ctor, nz, ngf, hw, bsz, dev):
    from damc import synth
    from src import diffusion_net as dn

    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(dev).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(71, 0, (bsz, 3, hw, hw))).to(dev)
    z0 = torch.from_numpy(synth.normal_f32(72, 0, (bsz, nz))).to(dev)
    p0 = torch.cat([z0, torch.from_numpy(synth.normal_f32(73, 0, (bsz, nz))).to(dev)])
    return G, E, x, z0, p0


def _block_vs_shards(G, E, x, z0, p0, post_steps, prior_steps, sigma):
    from damc import dist as ddist
    from damc import langevin as lv

    bsz = len(z0)
    za, pa = z0.clone(), p0.clone()
    lv.posterior_langevin(za, x, G, E, post_steps, sigma, 0.1, True, seed=31)
    lv.prior_langevin(pa, E, prior_steps, 0.4, True, seed=32, global_batch=2 * bsz)
    zs, ps = [], []
    for r in range(WORLD):
        pl = ddist.block_plan(bsz, r, WORLD, "strong")
        s, c, qs, qc = pl["post_start"], pl["post_count"], pl["prior_start"], pl["prior_count"]
        assert (c, qc) == (bsz // WORLD, 2 * bsz // WORLD)
        zb = z0[s:s + c].clone()
        lv.posterior_langevin(zb, x[s:s + c].contiguous(), G, E, post_steps, sigma, 0.1, True, seed=31, chain_base=s)
        pb = p0[qs:qs + qc].clone()
        lv.prior_langevin(pb, E, prior_steps, 0.4, True, seed=32, chain_base=qs, global_batch=pl["prior_global"])
        zs.append(zb)
        ps.append(pb)
    torch.cuda.synchronize()
    assert torch.isfinite(za).all() and torch.isfinite(pa).all() and not torch.equal(za, z0)
    zc, pc = torch.cat(zs), torch.cat(ps)
    nd = int((zc != za).any(dim=1).sum())
    assert torch.equal(zc, za), "%d of %d posterior chains differ between the block and its %d shards" % (
        nd, bsz, WORLD)
    assert torch.equal(pc, pa), "prior chains differ between the block and its %d shards" % WORLD


def test_cifar10_b128_block_is_bitwise_its_8_rank_shards(gpu_device):
    """The headline block (30 posterior steps on B=128 + 60 prior steps on 2B=256, in-kernel Philox noise) against
    8 ranks' slices of 16 posterior / 32 prior chains."""
    G, E, x, z0, p0 = _gen_case("_netG_cifar10", 128, 128, 32, 128, gpu_device)
    _block_vs_shards(G, E, x, z0, p0, 30, 60, 0.1)


def test_celeba64_b256_block_is_bitwise_its_8_rank_shards(gpu_device):
    """BASELINE config 4 (CelebA-64, nz=100, B=256 over 8 GPUs): 8 slices of 32 posterior / 64 prior chains."""
    G, E, x, z0, p0 = _gen_case("_netG_celeba64", 100, 128, 64, 256, gpu_device)
    _block_vs_shards(G, E, x, z0, p0, 10, 20, 0.1)


def test_celebaHQ_q_forward_b64_is_bitwise_its_8_rank_sweeps(gpu_device):
    """BASELINE config 5's named workload, Q(x) = Encoder_celebaHQ + the 100-step reverse sweep, at B=64 in one call
    against 8 calls of B=8 (each its slice of x and of the initial zt, the global seed, chain_base = the slice start).
    The team sweep partitions row tiles over the teams by the batch (B=8: one team holds rows), and the encoder runs
    split-K at B=8 and unsplit at B=64, so this pins both partitions to the same per-row arithmetic."""
    from damc import amortizer, synth
    from src import diffusion_net as dn

    Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset="celebaHQ")
    synth.load_into(Q, 20)
    Q.to(gpu_device).eval()
    x = torch.from_numpy(synth.uniform_f32(81, 0, (64, 3, 256, 256))).to(gpu_device)
    zt0 = torch.from_numpy(synth.normal_f32(82, 0, (64, 128))).to(gpu_device)
    with torch.no_grad():
        za = amortizer.q_forward(Q, x=x, zt=zt0, seed=9)
        parts = [amortizer.q_forward(Q, x=x[8 * r:8 * r + 8].contiguous(), zt=zt0[8 * r:8 * r + 8], seed=9,
                                     chain_base=8 * r) for r in range(WORLD)]
    torch.cuda.synchronize()
    zc = torch.cat(parts)
    assert torch.isfinite(za).all() and not torch.equal(za, zt0)
    nd = int((zc != za).any(dim=1).sum())
    assert torch.equal(zc, za), "%d of 64 sweep rows differ between B=64 and 8 x B=8" % nd


def test_bench_eight_ranks_union_is_the_one_rank_block(tmp_path, gpu_device):
    """`python bench.py --gpus 8` (the driver's 8-GPU command form), its 8 ranks sharing this GPU over gloo: the
    union of the ranks' final posterior and prior chains is bitwise the 1-rank block, and the JSON line reports the
    8-rank strong-scaling configuration (16 posterior / 32 prior chains per rank)."""
    one, eight = tmp_path / "one", tmp_path / "eight"
    one.mkdir()
    eight.mkdir()
    _run(one, 1, "strong")
    j8 = _run(eight, WORLD, "strong", extra_args=["--no-weak-extra"], timeout=420)
    assert j8["n_gpus"] == WORLD and j8["scaling"] == "strong"
    assert j8["config"]["global_batch"] == 128 and j8["config"]["per_rank_batch"] == 16
    assert j8["config"]["per_rank_prior_chains"] == 32 and j8["value"] > 0
    ref = torch.load(one / "rank0.pt", weights_only=True)
    parts = [torch.load(eight / ("rank%d.pt" % r), weights_only=True) for r in range(WORLD)]
    assert [p["plan"]["post_start"] for p in parts] == list(np.arange(WORLD) * 16)
    assert [p["plan"]["prior_start"] for p in parts] == list(np.arange(WORLD) * 32)
    assert torch.equal(torch.cat([p["z"] for p in parts]), ref["z"])
    assert torch.equal(torch.cat([p["p"] for p in parts]), ref["p"])
