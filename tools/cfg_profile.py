#!/usr/bin/env python
"""One BASELINE config's generator at a given batch (bench.py CONFIG_LEGS shapes): posterior Langevin steps for
rocprofv3 --kernel-trace (which launches bound a config leg).  usage: cfg_profile.py CTOR NZ NGF HW B [STEPS]"""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diffusion-amortized-mcmc_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import bench  # noqa: E402
from damc import langevin as lv  # noqa: E402
from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

ctor, nz, ngf, hw, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
steps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
dev = torch.device("cuda:0")
G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(dev).eval()
E = synth.load_into(dn._netE(nz=nz), 10).to(dev).eval()
x = torch.from_numpy(synth.uniform_f32(61, 0, (B, 3, hw, hw))).to(dev)
z = torch.from_numpy(synth.normal_f32(62, 0, (B, nz))).to(dev)
lv.posterior_langevin(z, x, G, E, steps, 1.0, 0.1, True, seed=9)
torch.cuda.synchronize()
ms = bench.event_ms(lambda: lv.posterior_langevin(z, x, G, E, steps, 1.0, 0.1, True, seed=9), reps=2) / steps
print("%s B=%d: %.3f ms per posterior step" % (ctor, B, ms))
