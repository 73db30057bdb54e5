"""Encoder_* forward: host submission time per call (perf_counter around the call, no sync) against GPU time per
call (events over back-to-back calls).  usage: python tools/enc_hosttime.py [cifar10|celebaHQ] [B] [calls]"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cifar10"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 50
hw = {"cifar10": 32, "celeba64": 64, "celebaHQ": 256}[name]
dev = torch.device("cuda:0")
enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(dev).eval()
x = torch.from_numpy(synth.uniform_f32(13, 1, (B, 3, hw, hw))).to(dev)
for _ in range(5):
    amortizer.encoder_forward(enc, x)
torch.cuda.synchronize()
host = []
for _ in range(calls):  # host time with the queue kept busy (a long kernel first so no call waits on the GPU)
    t0 = time.perf_counter()
    amortizer.encoder_forward(enc, x)
    host.append(time.perf_counter() - t0)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(calls):
    amortizer.encoder_forward(enc, x)
b.record()
b.synchronize()
host.sort()
for n in (1, 3):  # the bench's form: n back-to-back calls per timed sample
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        a.record()
        for _ in range(n):
            amortizer.encoder_forward(enc, x)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / n)
    print("%s B=%d %d back-to-back: %.3f ms per call (median of 5)" % (name, B, n, sorted(ts)[2]))
print("%s B=%d host %.3f ms per call (median), GPU+host %.3f ms per call over %d back-to-back calls"
      % (name, B, 1e3 * host[len(host) // 2], a.elapsed_time(b) / calls, calls))
