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
    q.put((rank, mse, mu, sigma))
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
        assert abs(mse - want_mse) < 1e-12
        assert torch.allclose(mu, want_mu, atol=1e-12)
        assert torch.allclose(sigma, want_sigma, atol=1e-10)
