#!/usr/bin/env python
"""One 60-step prior chain per engine at B = 16384 chains (CIFAR _netE, nz 128, nh 200): the workload of
rocprofv3 --pmc passes (MFMA busy cycles of prior_chain_mfma_kernel vs the VALU kernel) and of the kernel trace."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diffusion-amortized-mcmc_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import bench  # noqa: E402
from damc import langevin as lv  # noqa: E402

dev = torch.device("cuda:0")
G, E = bench.build(dev)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
z = torch.randn(B, 128, device=dev)
for engine in ("valu", "mfma"):
    zz = z.clone()
    lv.prior_langevin(zz, E, 60, 0.4, True, seed=3, engine=engine)
torch.cuda.synchronize()
flops = 4.0 * B * 60 * (128 * 200 + 200 * 200)
for engine in ("valu", "mfma"):
    ms = bench.event_ms(lambda: lv.prior_langevin(z.clone(), E, 60, 0.4, True, seed=3, engine=engine), reps=3)
    print("%s: B=%d x 60 steps %.3f ms, %.1f TFLOP/s fp32 (%.2f of the 157.3 fp32 MFMA / VALU peak)"
          % (engine, B, ms, flops / ms / 1e9, flops / ms / 1e9 / 157.3))
