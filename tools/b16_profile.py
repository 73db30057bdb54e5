#!/usr/bin/env python
"""The headline generator at a strong-scaling per-rank batch (CIFAR-10 ngf=128, B=16 by default): 10 posterior
steps, for rocprofv3 --kernel-trace --stats (which kernels bound the small per-rank batch)."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diffusion-amortized-mcmc_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import bench  # noqa: E402
from damc import langevin as lv  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
G, E = bench.build(dev)
x = torch.rand(B, 3, 32, 32, device=dev) * 2 - 1
z = torch.randn(B, 128, device=dev)
for _ in range(3):
    lv.posterior_langevin(z, x, G, E, 10, 0.1, 0.1, True, seed=1)
torch.cuda.synchronize()
ms = bench.event_ms(lambda: lv.posterior_langevin(z, x, G, E, 10, 0.1, 0.1, True, seed=1), reps=3) / 10
print("B=%d: %.3f ms per posterior step" % (B, ms))
