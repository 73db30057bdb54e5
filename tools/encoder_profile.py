"""Encoder_* forward (a10) for rocprofv3 --kernel-trace --stats: CIFAR-10 nif=64 at B=128 and CelebA-HQ nif=64 at B=64,
a few calls each.  usage: python tools/encoder_profile.py [cifar10|celebaHQ] [B] [calls]"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cifar10"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 5
hw = {"cifar10": 32, "celeba64": 64, "celebaHQ": 256}[name]
dev = torch.device("cuda:0")
enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(dev).eval()
x = torch.from_numpy(synth.uniform_f32(13, 1, (B, 3, hw, hw))).to(dev)
for _ in range(calls):
    amortizer.encoder_forward(enc, x)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(calls):
    amortizer.encoder_forward(enc, x)
b.record()
b.synchronize()
print("%s B=%d encoder %.3f ms per call" % (name, B, a.elapsed_time(b) / calls))
