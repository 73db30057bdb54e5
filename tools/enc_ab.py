"""Encoder_* forward (a10) time over one env switch, interleaved: usage: python tools/enc_ab.py VAR v1,v2 net:B ...
e.g. DAMC_ENC_FIRST_MFMA 1,0 celebaHQ:64 celebaHQ:8 (nif 64, nemb 1024; three back-to-back calls per sample)"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

var, vals = sys.argv[1], sys.argv[2].split(",")
dev = torch.device("cuda:0")
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for case in sys.argv[3:]:
    name, B = case.split(":")[0], int(case.split(":")[1])
    hw = {"cifar10": 32, "celeba64": 64, "celebaHQ": 256}[name]
    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 1, (B, 3, hw, hw))).to(dev)
    outs = {}
    for r in range(2):
        for v in vals:
            os.environ[var] = v
            outs[v] = amortizer.encoder_forward(enc, x).clone()
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                a.record()
                for _ in range(3):
                    amortizer.encoder_forward(enc, x)
                b.record()
                b.synchronize()
                ts.append(a.elapsed_time(b) / 3)
            print("%s B=%d %s=%s %.4f ms per call (median of 5)" % (name, B, var, v, sorted(ts)[2]), flush=True)
    ref = outs[vals[-1]].double()
    for v in vals[:-1]:
        d = float((outs[v].double() - ref).norm() / ref.norm())
        print("%s B=%d xemb rel-L2 %s=%s vs %s: %.2e" % (name, B, var, v, vals[-1], d), flush=True)
    del enc, x
    torch.cuda.empty_cache()
