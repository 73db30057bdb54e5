#!/usr/bin/env python
"""Q(x) sweep at B=128 (CIFAR defaults) for rocprofv3 --kernel-trace --stats."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diffusion-amortized-mcmc_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
bench.B = B
print(bench.amortizer_bench(torch.device("cuda:0")))
