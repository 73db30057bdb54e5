#!/usr/bin/env python
"""Prior chain (60 steps on 2B=256 chains) and posterior update timing at the CIFAR-10 bench config."""
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
for nchains in (256, 128, 512, 1024, 2048, 4096, 16384):
    z = torch.randn(nchains, 128, device=dev)
    res = []
    for engine in ("valu", "mfma"):
        def prior():
            lv.prior_langevin(z, E, 60, 0.4, True, seed=3, engine=engine)

        ms = bench.event_ms(prior, reps=5)
        res.append("%s %.3f ms = %.2f us/step" % (engine, ms, 1e3 * ms / 60))
    print("prior chain: %5d chains x 60 steps: %s" % (nchains, "  |  ".join(res)))
x = torch.rand(128, 3, 32, 32, device=dev) * 2 - 1
z = torch.randn(128, 128, device=dev)
from damc import _lib  # noqa: E402
import ctypes  # noqa: E402

L = _lib.lib()
L.damc_prof_reset()
L.damc_prof_select(b"posterior_update,prior_chain")
L.damc_prof_enable(1)
for _ in range(3):
    lv.posterior_langevin(z, x, G, E, 10, 0.1, 0.1, True, seed=4)
    lv.prior_langevin(torch.randn(256, 128, device=dev), E, 60, 0.4, True, seed=3)
torch.cuda.synchronize()
L.damc_prof_enable(0)
for name in (b"posterior_update", b"prior_chain"):
    t, n, f = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
    L.damc_prof_query(name, ctypes.byref(t), ctypes.byref(n), ctypes.byref(f))
    if n.value:
        print("%s: %d launches, %.2f us per launch" % (name.decode(), n.value, 1e3 * t.value / n.value))
