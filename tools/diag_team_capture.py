"""Round 2's graph-replay timeout of the team sweep, reproduced and explained: capture the team launch with the flags
zeroed by a hipMemsetAsync node (DAMC_SWEEP_MEMSET_FLAGS=1, round 2's form) and with the setup kernel zeroing them
(default), replay each, and print per form: bitwise vs eager, the rescue count, and the control words of the last
replay (which team slots had published which stage; the failed waits' {stage needed, first late flag, late mask})."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib  # noqa: E402
from damc import amortizer as am  # noqa: E402
from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

os.environ["DAMC_SWEEP_TEAM_KEEP"] = "1"
os.environ["DAMC_SWEEP_SENT"] = "0"  # the flag protocol (round 2's): the data-driven default polls no flags
dev = torch.device("cuda:0")
n, B = 20, 128
Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=n, logsnr_min=-5.1,
               logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
synth.load_into(Q, 20)
Q.to(dev).eval()
xemb = torch.from_numpy(synth.normal_f32(7, 0, (B, 1024))).to(dev)
zt0 = torch.from_numpy(synth.normal_f32(8, 0, (B, 128))).to(dev)
L = _lib.lib()
ze = zt0.clone()
am.reverse_sweep(Q, xemb, ze, seed=42)
torch.cuda.synchronize()
plan = am._DEN[Q.p]
for form in ("memset node (round 2)", "setup kernel (round 3)"):
    os.environ["DAMC_SWEEP_MEMSET_FLAGS"] = "1" if form.startswith("memset") else "0"
    before = L.damc_sweep_team_failures(0)
    zg = zt0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        am.reverse_sweep(Q, xemb, zg.clone(), seed=42)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        am.reverse_sweep(Q, xemb, zg, seed=42)
    same = []
    for _ in range(3):
        zg.copy_(zt0)
        g.replay()
        torch.cuda.synchronize()
        same.append(bool(torch.equal(zg, ze)))
    fails = L.damc_sweep_team_failures(0) - before
    d = plan.pack(dev)
    ws = plan._ws._tls.ws[1]  # the workspace the capture recorded (the cache's last entry; the replays use it)
    nbytes = int(L.damc_sweep_workspace_bytes(ctypes.byref(d), B, n))
    words = np.zeros(8 * 64 * 32 + 64 + 8 * 64 * 4, dtype=np.int32)
    _lib.check(L.damc_sweep_team_words(ctypes.byref(d), B, n, _lib.ptr(ws), nbytes,
                                       words.ctypes.data_as(ctypes.c_void_p), words.size), "team words")
    flags = words[:8 * 64 * 32].reshape(8, 64, 32)[:, :, 0]
    err = words[8 * 64 * 32]
    diag = words[8 * 64 * 32 + 64:].reshape(-1, 4)
    print("%s: replays bitwise = %s, rescued replays = %d, error word = %d" % (form, same, fails, err))
    print("  stages published per team (min / max over its 32 slots):",
          [(int(flags[t, :32].min()), int(flags[t, :32].max())) for t in range(8)])
    bad = [(i, list(map(int, r))) for i, r in enumerate(diag) if r[0]]
    print("  failed waits (workgroup, [stage needed, first late flag, late mask lo, hi]): %d, first %s"
          % (len(bad), bad[:6]))
    del g
