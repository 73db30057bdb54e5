"""A/B of team-sweep variants selected by environment variables read per call (interleaved, one process): per variant
the median sweep time and whether the result is bitwise the first variant's.  CIFAR-10 Q: nif 64, nxemb 1024, ntemb
128, 100 steps, B=128 (or argv[1]).  usage: python tools/sweep_ab.py [B] [VAR=val,VAR=val ...] ..."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib, amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
variants = sys.argv[2:] or ["DAMC_SWEEP_SENT=0", "DAMC_SWEEP_SENT=1"]
dev = torch.device("cuda:0")
Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100, logsnr_min=-5.1,
               logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
synth.load_into(Q, 20)
Q.to(dev).eval()
xemb = torch.from_numpy(synth.normal_f32(7, 0, (B, 1024))).to(dev)
zt0 = torch.from_numpy(synth.normal_f32(8, 0, (B, 128))).to(dev)


def setenv(v):
    for kv in v.split(","):
        k, val = kv.split("=")
        os.environ[k] = val


times = {v: [] for v in variants}
res = {}
for rep in range(7):
    for v in variants:
        setenv(v)
        z = zt0.clone()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        amortizer.reverse_sweep(Q, xemb, z, seed=11)
        b.record()
        b.synchronize()
        times[v].append(a.elapsed_time(b))
        res[v] = z
        for kv in v.split(","):
            os.environ.pop(kv.split("=")[0], None)
ref = res[variants[0]]
for v in variants:
    t = sorted(times[v])[len(times[v]) // 2]
    print("%-40s B=%d sweep %.3f ms (%.2f us/step)  bitwise=%s  finite=%s  rescues=%d" % (
        v, B, t, 10 * t, bool(torch.equal(res[v], ref)), bool(torch.isfinite(res[v]).all()),
        _lib.lib().damc_sweep_team_failures(0)))
