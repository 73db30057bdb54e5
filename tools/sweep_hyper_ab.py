"""Reverse sweep (CIFAR Q, B=128, 100 steps, the bench's config) wall time per call over DAMC_SWEEP_HYPER (limb /
fp32), interleaved; three back-to-back calls per sample as in bench.py.  usage: python tools/sweep_hyper_ab.py [reps] [mode,...]  (mode: limb / fp32, or VAR=value)"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100,
               logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
               dataset="cifar10")
synth.load_into(Q, 20)
Q.to(dev).eval()
for p in Q.parameters():
    p.requires_grad_(False)
xemb = torch.from_numpy(synth.normal_f32(31, 0, (128, 1024))).to(dev)
zt = torch.from_numpy(synth.normal_f32(32, 0, (128, 128))).to(dev)
zw = torch.empty_like(zt)


def sweep():
    zw.copy_(zt)
    amortizer.reverse_sweep(Q, xemb, zw, seed=5)


a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(reps):
    for mode in sys.argv[2].split(",") if len(sys.argv) > 2 else ("limb", "fp32"):
        var, _, val = mode.partition("=")
        if not val:  # a bare mode name: DAMC_SWEEP_HYPER
            var, val = "DAMC_SWEEP_HYPER", mode
        os.environ[var] = val
        sweep()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            a.record()
            for _ in range(3):
                sweep()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) / 3)
        ms = sorted(ts)[2]
        print("hyper=%s sweep %.3f ms per call, %.2f us per denoise step" % (mode, ms, 10 * ms), flush=True)
