#!/usr/bin/env python
"""Host time of the Q update's pieces (tools/q_update_trace.py's step) without cProfile's per-call overhead: the
autograd Functions' forward / backward (the backward ones run on autograd's device thread, which cProfile does not
see), prior_emb, the optimiser, and the whole step, as perf_counter sums over `calls` updates after 3 warm-ups.
usage: python tools/q_update_hosttime.py [calls]"""
import collections
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch  # noqa: E402

from damc import optim as dopt  # noqa: E402
from damc import synth, training  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 50
B, NZ = 128, 128
dev = torch.device("cuda:0")
Q = dn._netQ_U(nc=3, nz=NZ, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100, logsnr_min=-5.1,
               logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A", dataset="cifar10")
synth.load_into(Q, 20)
Q.to(dev).train()
opt = dopt.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
x = torch.from_numpy(synth.uniform_f32(51, 0, (B, 3, 32, 32))).to(dev)
z = torch.from_numpy(synth.normal_f32(52, 0, (B, NZ))).to(dev)
mask = (torch.from_numpy(synth.uniform_f32(53, 0, (B, 1), 0.0, 1.0)) >= 0.2).float().to(dev)
acc = collections.Counter()


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        acc[name] += time.perf_counter() - t0
        return r
    return w


for cls, nm in ((training._EncoderTrainFn, "encoder"), (training._DenoiserTrainFn, "denoiser"),
                (training._QLossFn, "loss")):
    cls.forward = staticmethod(timed(nm + ".forward", cls.forward))
    cls.backward = staticmethod(timed(nm + ".backward", cls.backward))
Q.prior_emb.forward = timed("prior_emb.forward", Q.prior_emb.forward)
training.q_noise_glue = timed("q_noise_glue", training.q_noise_glue)
opt.clip_and_step = timed("clip_and_step", opt.clip_and_step)


def step():
    t0 = time.perf_counter()
    opt.zero_grad(set_to_none=True)
    t1 = time.perf_counter()
    loss = Q.calculate_loss(x=x, z=z, mask=mask).mean()
    t2 = time.perf_counter()
    loss.backward()
    t3 = time.perf_counter()
    opt.clip_and_step(100)
    acc["zero_grad"] += t1 - t0
    acc["calculate_loss+mean"] += t2 - t1
    acc["backward()"] += t3 - t2
    acc["step"] += time.perf_counter() - t0


for _ in range(3):
    step()
torch.cuda.synchronize()
acc.clear()
for _ in range(calls):
    step()
torch.cuda.synchronize()
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print("%-22s %7.3f ms per update" % (k, v * 1e3 / calls))
