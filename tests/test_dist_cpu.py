"""CPU, world_size 2 over gloo: sharding covers the batch exactly once and the final statistic
reductions (recon MSE, FID sufficient statistics) equal the single-process results."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from damc import dist as ddist


def test_shard_partition():
    for gb in (1, 7, 64, 128, 130, 256):
        for world in (1, 2, 3, 4, 8):
            covered = []
            for r in range(world):
                s, c = ddist.shard(gb, r, world)
                covered += list(range(s, s + c))
            assert covered == list(range(gb))
    assert ddist.shard(128, 3, 8) == (48, 16)
    with pytest.raises(ValueError):
        ddist.shard(8, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as d

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    d.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(10, 3, 4, 4, generator=g)
    xh = torch.rand(10, 3, 4, 4, generator=g)
    feats = torch.randn(10, 6, generator=g)
    s, c = ddist.shard(10, rank, world)
    m = ddist.ReconMSE(torch.device("cpu"))
    m.update(xh[s:s + c], x[s:s + c])
    f = ddist.FidStats(6, torch.device("cpu"))
    f.update(feats[s:s + c])
    mse = m.compute()
    mu, sigma = f.compute()
    # numpy copies: a tensor on a spawn queue is a shared-memory handle that dies with this process
    q.put((rank, mse, mu.numpy().copy(), sigma.numpy().copy()))
    d.destroy_process_group()


def test_reductions_match_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = torch.Generator().manual_seed(0)
    x = torch.rand(10, 3, 4, 4, generator=g)
    xh = torch.rand(10, 3, 4, 4, generator=g)
    feats = torch.randn(10, 6, generator=g).double()
    want_mse = float(((xh - x) ** 2).mean(dim=(1, 2, 3)).double().mean())
    want_mu = feats.mean(0)
    want_sigma = torch.cov(feats.t())
    for _, mse, mu, sigma in res:
        mu, sigma = torch.from_numpy(mu), torch.from_numpy(sigma)
        assert abs(mse - want_mse) < 1e-12
        assert torch.allclose(mu, want_mu, atol=1e-12)
        assert torch.allclose(sigma, want_sigma, atol=1e-10)


def _plan_worker(rank, world, port, q):
    """One rank of a strong-scaling bench block: its plan and its slices of the global inputs."""
    import sys

    import torch.distributed as d

    from conftest import REPO

    sys.path.insert(0, REPO)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    d.init_process_group("gloo", rank=rank, world_size=world)
    plan = ddist.block_plan(bench.B, rank, world, "strong")
    x, z0, p0 = bench.inputs(torch.device("cpu"), rank, plan, "strong")
    # reassemble on every rank: gather the per-rank row counts, then the padded slices
    counts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    d.all_gather(counts, torch.tensor([plan["post_count"], plan["prior_count"]]))
    pad = lambda t, n: torch.cat([t, t.new_zeros((n - t.shape[0],) + tuple(t.shape[1:]))])  # noqa: E731
    mx, mq = max(int(c[0]) for c in counts), max(int(c[1]) for c in counts)
    gx = [torch.empty((mx,) + tuple(x.shape[1:])) for _ in range(world)]
    gz = [torch.empty(mx, z0.shape[1]) for _ in range(world)]
    gp = [torch.empty(mq, p0.shape[1]) for _ in range(world)]
    d.all_gather(gx, pad(x, mx))
    d.all_gather(gz, pad(z0, mx))
    d.all_gather(gp, pad(p0, mq))
    bases = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    d.all_gather(bases, torch.tensor([plan["post_start"], plan["prior_start"]]))
    if rank == 0:
        n = [(int(c[0]), int(c[1])) for c in counts]
        q.put((torch.cat([g[:c] for g, (c, _) in zip(gx, n)]).numpy(), torch.cat([g[:c] for g, (c, _) in zip(gz, n)]).numpy(),
               torch.cat([g[:c] for g, (_, c) in zip(gp, n)]).numpy(), [tuple(int(v) for v in b) for b in bases], n))
    d.destroy_process_group()


def test_strong_scaling_plan_reassembles_the_global_block():
    """bench.py --scaling strong over gloo, world 2: the ranks' slices of x / z0 / the prior chains
    concatenate to the global B=128 block (2B = 256 prior chains = cat(z0, N(0, I))), and each rank's Philox
    chain_base is the global index of its first chain, so noise streams are those of the 1-GPU block."""
    import sys

    from conftest import REPO

    sys.path.insert(0, REPO)
    import bench

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    x, z0, p0, bases, counts = q.get(timeout=180)
    x, z0, p0 = (torch.from_numpy(a) for a in (x, z0, p0))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    plan1 = ddist.block_plan(bench.B, 0, 1, "strong")
    gx, gz, gp = bench.inputs(torch.device("cpu"), 0, plan1, "strong")
    assert torch.equal(x, gx) and torch.equal(z0, gz) and torch.equal(p0, gp)
    assert gp.shape[0] == 2 * bench.B and torch.equal(gp[:bench.B], gz)
    assert bases == [(0, 0), (counts[0][0], counts[0][1])]
    assert sum(c for c, _ in counts) == bench.B and sum(c for _, c in counts) == 2 * bench.B
    weak = [ddist.block_plan(bench.B, r, 4, "weak") for r in range(4)]
    assert [w["post_start"] for w in weak] == [0, 128, 256, 384]
    assert [w["prior_start"] for w in weak] == [0, 256, 512, 768]


def test_bench_gpus_n_launches_n_ranks_without_a_launcher():
    """`python bench.py --gpus 2` (the driver's command form, no torchrun around it) starts 2 ranks itself: they
    rendezvous (gloo, --dry-run: no GPU here) and see a world of 2; strong scaling splits the global B=128."""
    import json
    import subprocess
    import sys

    from conftest import REPO

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert j["n_gpus"] == 2 and j["scaling"] == "strong"
    assert [p["post_count"] for p in j["plans"]] == [64, 64]
    assert [p["prior_start"] for p in j["plans"]] == [0, 128]
    assert all(p["prior_global"] == 256 for p in j["plans"])


def test_bench_refuses_a_world_that_disagrees_with_gpus():
    import subprocess
    import sys

    from conftest import REPO

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--dry-run"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus 3" in r.stderr
