"""The multi-GPU path of bench.py end to end on one MI355X: `python bench.py --gpus 2` (no launcher around it, the
driver's command form) starts two ranks itself; they share the GPU over the gloo backend (RCCL needs one GPU per rank; the driver's 8-GPU runs use nccl = RCCL).  Each rank runs
its slice of the BASELINE Langevin block on the HIP path (damc.dist.block_plan, chain_base = the slice start) and
the ranks' timings go through the MAX all-reduce.  Checks: the JSON line's multi-rank fields, and — strong
scaling — the union of the two ranks' chains is bitwise the 1-rank block (posterior and prior chains), because
the Philox noise is keyed by the global chain index and nothing else couples the chains."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp, world, scaling, torchrun=False, backend="gloo", extra_args=(), timeout=240, **extra_env):
    os.makedirs(tmp, exist_ok=True)
    env = dict(os.environ, DAMC_DIST_BACKEND=backend, DAMC_BENCH_DUMP=str(tmp), **extra_env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    args = ["bench.py", "--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-extras", "--no-cpu-baseline",
            "--scaling", scaling] + list(extra_args)
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=HERE, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_two_ranks_strong_scaling_union_is_the_one_rank_block(tmp_path, gpu_device):
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    j1 = _run(one, 1, "strong")
    j2 = _run(two, 2, "strong")
    assert j2["n_gpus"] == 2 and j2["scaling"] == "strong"
    assert j2["config"]["global_batch"] == 128 and j2["config"]["per_rank_batch"] == 64
    assert j2["weak_scaling"]["per_rank_batch"] == 128 and j2["weak_scaling"]["global_batch"] == 256
    assert j2["per_rank"]["avg_launch_ms_max_over_ranks"] > 0
    assert j2["value"] > 0 and j1["value"] > 0
    ref = torch.load(one / "rank0.pt", weights_only=True)
    parts = [torch.load(two / ("rank%d.pt" % r), weights_only=True) for r in range(2)]
    assert [p["plan"]["post_start"] for p in parts] == [0, 64]
    assert [p["plan"]["prior_start"] for p in parts] == [0, 128]
    z = torch.cat([p["z"] for p in parts])
    pz = torch.cat([p["p"] for p in parts])
    assert torch.isfinite(z).all() and torch.isfinite(pz).all()
    assert torch.equal(z, ref["z"]), "posterior chains of the 2-rank block differ from the 1-rank block"
    assert torch.equal(pz, ref["p"]), "prior chains of the 2-rank block differ from the 1-rank block"


def test_strong_scaling_union_keeps_the_prior_engine_of_the_global_block(tmp_path, gpu_device):
    """the prior engine is chosen from the GLOBAL chain count.  With the MFMA threshold at 200 the
    1-rank block (256 prior chains) runs the MFMA engine; each rank of 2 holds 128 chains and must run it too, or
    the union is no longer bitwise the 1-rank block."""
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    _run(one, 1, "strong", DAMC_EBM_MFMA_MIN_B="200")
    _run(two, 2, "strong", DAMC_EBM_MFMA_MIN_B="200")
    ref = torch.load(one / "rank0.pt", weights_only=True)
    parts = [torch.load(two / ("rank%d.pt" % r), weights_only=True) for r in range(2)]
    assert torch.equal(torch.cat([p["p"] for p in parts]), ref["p"])
    assert torch.equal(torch.cat([p["z"] for p in parts]), ref["z"])


def test_two_ranks_weak_scaling_line(tmp_path, gpu_device):
    j = _run(tmp_path, 2, "weak", torchrun=True)
    assert j["n_gpus"] == 2 and j["scaling"] == "weak"
    assert j["config"]["per_rank_batch"] == 128
    parts = [torch.load(tmp_path / ("rank%d.pt" % r), weights_only=True) for r in range(2)]
    assert [p["plan"]["post_start"] for p in parts] == [0, 128]
    # distinct global chains: the two ranks' noise streams differ, so their chains do too
    assert not torch.equal(parts[0]["z"], parts[1]["z"])


def test_one_rank_over_rccl_is_the_plain_block(tmp_path, gpu_device):
    """RCCL itself on a one-GPU box: bench.py under torch.distributed.run with one rank and backend nccl (RCCL), the
    process group forced on (DAMC_BENCH_PG=1) so its barrier and MAX all-reduce run over RCCL; the rank's chains are
    bitwise the plain single-process block (no collective touches the data path)."""
    j = _run(tmp_path / "rccl", 1, "strong", torchrun=True, backend="nccl", DAMC_BENCH_PG="1")
    ref = _run(tmp_path / "plain", 1, "strong")
    assert j["n_gpus"] == 1 and j["value"] > 0
    a = torch.load(tmp_path / "rccl" / "rank0.pt", weights_only=True)
    b = torch.load(tmp_path / "plain" / "rank0.pt", weights_only=True)
    assert torch.equal(a["z"], b["z"]) and torch.equal(a["p"], b["p"])
