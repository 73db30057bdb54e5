"""Posterior step time (CIFAR-10 _netG_cifar10 ngf=128 + _netE, sigma 0.1, noise on) over one env switch, interleaved:
usage: python tools/post_step_ab.py VAR v1,v2 [B ...]   e.g. DAMC_X3_SKINNY 1,0 128 64"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import langevin as lv, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

var, vals = sys.argv[1], sys.argv[2].split(",")
Bs = [int(b) for b in sys.argv[3:]] or [128]
dev = torch.device("cuda:0")
G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0).to(dev).eval()
E = synth.load_into(dn._netE(nz=128), 10).to(dev).eval()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for B in Bs:
    x = torch.from_numpy(synth.uniform_f32(61, 0, (B, 3, 32, 32))).to(dev)
    z0 = torch.from_numpy(synth.normal_f32(62, 0, (B, 128))).to(dev)
    z = torch.empty_like(z0)
    for r in range(2):
        for v in vals:
            os.environ[var] = v
            ts = []
            for _ in range(6):
                z.copy_(z0)
                torch.cuda.synchronize()
                a.record()
                lv.posterior_langevin(z, x, G, E, 10, 0.1, 0.1, True, seed=9)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) / 10)
            print("B=%d %s=%s %.4f ms per posterior step (median of 5 after 1)" % (B, var, v, sorted(ts[1:])[2]),
                  flush=True)
