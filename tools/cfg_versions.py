#!/usr/bin/env python
"""Posterior-step time of one library tree on the BASELINE generator configs and their per-rank batches (the bench's
config_legs plus the headline B=128): 10-step posterior calls with in-kernel noise, median of 7 event-timed calls after
2 warm-ups, per step, with a checksum of z so trees can be compared bitwise.  argv[1]: a checkout holding
diffusion-amortized-mcmc_amd/ with its own built libdamc.so (default: this repo); argv[2:]: leg names (default all).
usage: python tools/cfg_versions.py [tree] [leg ...]"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tree = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 and os.path.isdir(sys.argv[1]) else HERE
names = [a for a in sys.argv[1:] if not os.path.isdir(a)]
sys.path[:0] = [os.path.join(tree, "diffusion-amortized-mcmc_amd")]
import torch  # noqa: E402

from damc import langevin as lv  # noqa: E402
from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

LEGS = {  # name: (constructor, nz, ngf, image size, B, sigma)
    "cifar16": ("_netG_cifar10", 128, 128, 32, 16, 0.1),
    "cifar128": ("_netG_cifar10", 128, 128, 32, 128, 0.1),
    "svhn64": ("_netG_svhn", 100, 64, 32, 64, 0.1),
    "celeba32": ("_netG_celeba64", 100, 128, 64, 32, 0.1),
    "hq8": ("_netG_celebaHQ", 128, 128, 256, 8, 1.0),
    "celeba256": ("_netG_celeba64", 100, 128, 64, 256, 0.1),
    "hq64": ("_netG_celebaHQ", 128, 128, 256, 64, 1.0),
}
DEFAULT = ["cifar16", "cifar128", "svhn64", "celeba32", "hq8"]
dev = torch.device("cuda:0")
for name in names or DEFAULT:
    ctor, nz, ngf, hw, B, sigma = LEGS[name]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(dev).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(11, 0, (B, 3, hw, hw))).to(dev)
    z0 = torch.from_numpy(synth.normal_f32(12, 0, (B, nz))).to(dev)
    ts = []
    for rep in range(9):
        z = z0.clone()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        lv.posterior_langevin(z, x, G, E, 10, sigma, 0.1, True, seed=1)
        b.record()
        b.synchronize()
        if rep >= 2:
            ts.append(a.elapsed_time(b) / 10)
    ts.sort()
    h = hashlib.sha1(z.cpu().numpy().tobytes()).hexdigest()[:12]
    print("%-12s %-9s %s posterior step median %.4f ms (min %.4f max %.4f)  sha %s" % (
        os.path.basename(tree.rstrip("/")), name, os.environ.get("DAMC_X3_NEGK_RULE", "-"), ts[len(ts) // 2], ts[0], ts[-1], h), flush=True)
