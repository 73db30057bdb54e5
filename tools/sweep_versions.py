#!/usr/bin/env python
"""Reverse-sweep time of one library tree (the sweep-regression A/B of round 4): CIFAR-10 Q (nif 64, nxemb 1024,
ntemb 128, 100 steps) at B=128 on the tree given as argv[1] (a checkout holding diffusion-amortized-mcmc_amd/ with
its own built libdamc.so; default: this repo), median of 15 event-timed sweeps after 3 warm-ups, plus a checksum
of the result so trees can be compared bitwise.  Environment variables (DAMC_SWEEP_*) pass through.
usage: python tools/sweep_versions.py [tree] [B]"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else HERE
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
sys.path[:0] = [os.path.join(tree, "diffusion-amortized-mcmc_amd")]
import torch  # noqa: E402

from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

dev = torch.device("cuda:0")
Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100, logsnr_min=-5.1,
               logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
synth.load_into(Q, 20)
Q.to(dev).eval()
xemb = torch.from_numpy(synth.normal_f32(7, 0, (B, 1024))).to(dev)
zt0 = torch.from_numpy(synth.normal_f32(8, 0, (B, 128))).to(dev)
ts = []
for rep in range(18):
    z = zt0.clone()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    amortizer.reverse_sweep(Q, xemb, z, seed=11)
    b.record()
    b.synchronize()
    if rep >= 3:
        ts.append(a.elapsed_time(b))
ts.sort()
h = hashlib.sha1(z.cpu().numpy().tobytes()).hexdigest()[:12]
print("%s B=%d sweep median %.3f ms (min %.3f, max %.3f) = %.2f us/step  sha %s  env %s" % (
    os.path.basename(tree.rstrip("/")), B, ts[len(ts) // 2], ts[0], ts[-1], 10 * ts[len(ts) // 2], h,
    " ".join("%s=%s" % kv for kv in os.environ.items() if kv[0].startswith("DAMC_SWEEP"))))
