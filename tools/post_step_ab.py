"""Posterior step time (full-width generator + _netE, noise on) over one env switch, interleaved:
usage: python tools/post_step_ab.py VAR v1,v2 [CASE ...]   CASE = B (CIFAR-10) or net:B, net in cifar10 / svhn /
celeba64 / celebaHQ; e.g. DAMC_X3_FIXUP 1,0 16 svhn:64 celebaHQ:8"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import langevin as lv, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

NETS = {"cifar10": ("_netG_cifar10", 128, 128, 32, 0.1), "svhn": ("_netG_svhn", 100, 64, 32, 0.1),
        "celeba64": ("_netG_celeba64", 100, 128, 64, 0.1), "celebaHQ": ("_netG_celebaHQ", 128, 128, 256, 1.0)}
var, vals = sys.argv[1], sys.argv[2].split(",")
cases = [(c.split(":")[0], int(c.split(":")[1])) if ":" in c else ("cifar10", int(c)) for c in sys.argv[3:]] or \
    [("cifar10", 128)]
dev = torch.device("cuda:0")
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for net, B in cases:
    ctor, nz, ngf, hw, sigma = NETS[net]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(dev).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(61, 0, (B, 3, hw, hw))).to(dev)
    z0 = torch.from_numpy(synth.normal_f32(62, 0, (B, nz))).to(dev)
    z = torch.empty_like(z0)
    for r in range(2):
        for v in vals:
            os.environ[var] = v
            ts = []
            for _ in range(6):
                z.copy_(z0)
                torch.cuda.synchronize()
                a.record()
                lv.posterior_langevin(z, x, G, E, 10, sigma, 0.1, True, seed=9)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) / 10)
            print("%s B=%d %s=%s %.4f ms per posterior step (median of 5 after 1)" % (net, B, var, v,
                                                                                     sorted(ts[1:])[2]), flush=True)
    del G, E, x, z0, z
    torch.cuda.empty_cache()
