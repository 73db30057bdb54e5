#!/usr/bin/env python
"""Posterior-step time of one library tree on the headline generator (CIFAR-10 ngf=128, nz=128): for each batch in
argv[2:] (default 16 128), 10-step posterior calls, median of 7 event-timed calls after 2 warm-ups, per step; plus a
checksum of z so trees can be compared bitwise.  argv[1]: a checkout holding diffusion-amortized-mcmc_amd/ with its
own built libdamc.so (default: this repo).  usage: python tools/step_versions.py [tree] [B ...]"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else HERE
Bs = [int(b) for b in sys.argv[2:]] or [16, 128]
sys.path[:0] = [os.path.join(tree, "diffusion-amortized-mcmc_amd")]
import torch  # noqa: E402

from damc import langevin as lv  # noqa: E402
from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

dev = torch.device("cuda:0")
G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0).to(dev).eval()
E = synth.load_into(dn._netE(nz=128), 10).to(dev).eval()
for B in Bs:
    x = torch.from_numpy(synth.uniform_f32(11, 0, (B, 3, 32, 32))).to(dev)
    z0 = torch.from_numpy(synth.normal_f32(12, 0, (B, 128))).to(dev)
    ts = []
    for rep in range(9):
        z = z0.clone()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        lv.posterior_langevin(z, x, G, E, 10, 0.1, 0.1, True, seed=1)
        b.record()
        b.synchronize()
        if rep >= 2:
            ts.append(a.elapsed_time(b) / 10)
    ts.sort()
    h = hashlib.sha1(z.cpu().numpy().tobytes()).hexdigest()[:12]
    print("%s B=%d posterior step median %.4f ms (min %.4f max %.4f)  sha %s" % (
        os.path.basename(tree.rstrip("/")), B, ts[len(ts) // 2], ts[0], ts[-1], h), flush=True)
