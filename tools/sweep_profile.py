#!/usr/bin/env python
"""Q(x) sweep at B=128 (CIFAR defaults): bench.amortizer_bench plus the per-class GPU time of one sweep from the
library's HIP-event profiler (denoise_chain = the 7n-launch dependent chain, sweep_pre / sweep_hyper = the
per-call GEMMs); also usable under rocprofv3 --kernel-trace --stats."""
import ctypes
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
from damc import _lib  # noqa: E402

L = _lib.lib()
names = ("denoise_chain", "sweep_pre", "sweep_hyper")
L.damc_prof_reset()
L.damc_prof_select(",".join(names).encode())
L.damc_prof_enable(1)
bench.amortizer_bench(torch.device("cuda:0"))
torch.cuda.synchronize()
L.damc_prof_enable(0)
for n in names:
    t, k, f = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
    L.damc_prof_query(n.encode(), ctypes.byref(t), ctypes.byref(k), ctypes.byref(f))
    if k.value:
        print("%s: %d launches, %.1f us per launch" % (n, k.value, 1e3 * t.value / k.value))
