#!/usr/bin/env python
"""Host-side profile of the Q update (tools/q_update_trace.py's step: Q.calculate_loss(...).mean().backward() +
damc.optim's fused clip + AdamW) at the bench config: cProfile over `calls` updates after 3 warm-up updates, the top
functions by own time and by cumulative time.  usage: python tools/q_update_hostprof.py [calls]"""
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch  # noqa: E402

from damc import optim as dopt  # noqa: E402
from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
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


def step():
    opt.zero_grad(set_to_none=True)
    Q.calculate_loss(x=x, z=z, mask=mask).mean().backward()
    opt.clip_and_step(100)


for _ in range(3):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(calls):
    step()
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(45)
