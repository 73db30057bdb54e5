"""Which encoder pre-activations sit on a LeakyReLU kink in a Q-update golden case: the encoder forward of the HIP
training path (its saved conv outputs y and InstanceNorm stats, a = ((y - mean) rstd) gamma + beta in fp64) against
an fp64 and an fp32 PyTorch forward of the same module and input; per InstanceNorm stage the sign disagreements and
the smallest |a|.  usage: python tools/diag_kink.py q_celebaHQ_s"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from conftest import build_q_case, load_golden  # noqa: E402

from damc import training  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "q_celebaHQ_s"
dev = torch.device("cuda:0")
rec, meta = load_golden(name + "_qtrain")
c = build_q_case(meta["q"], dev)
enc, x = c["Q"].encoder, c["x"]
enc.train()
cap = {}
orig = training._EncoderTrainFn.forward


def fwd(ctx, xx, stages, *params):
    r = orig(ctx, xx, stages, *params)
    cap["saved"], cap["stages"] = ctx.saved, ctx.stages
    return r


training._EncoderTrainFn.forward = staticmethod(fwd)
enc(x)
training._EncoderTrainFn.forward = staticmethod(orig)


def torch_pre(dt):
    h = x.to(dt)
    pres = []
    for conv, norm, slope in cap["stages"]:
        y = F.conv2d(h, conv.weight.to(dt), conv.bias.to(dt), conv.stride, conv.padding)
        if norm is None:
            break
        a = F.instance_norm(y, weight=norm.weight.to(dt), bias=norm.bias.to(dt), eps=norm.eps)
        pres.append(a)
        h = F.leaky_relu(a, slope)
    return pres


with torch.no_grad():
    p64, p32 = torch_pre(torch.float64), torch_pre(torch.float32)
for i, (conv, norm, slope) in enumerate(cap["stages"]):
    if norm is None:
        break
    h_in, y, stats, H, W, Ho, Wo = cap["saved"][i]
    st = stats.double().reshape(y.shape[0], -1, 2)
    a_h = ((y.double() - st[:, None, :, 0].reshape(y.shape[0], 1, 1, -1)) * st[:, :, 1].reshape(y.shape[0], 1, 1, -1)
           * norm.weight.double() + norm.bias.double())  # NHWC
    a64 = p64[i].permute(0, 2, 3, 1)
    a32 = p32[i].double().permute(0, 2, 3, 1)
    fh = ((a_h > 0) != (a64 > 0))
    f32 = ((a32 > 0) != (a64 > 0))
    print("stage %d (%dx%d, %d ch): sign flips hip vs fp64 %d, torch32 vs fp64 %d; min |a64| %.2e; |a64| at hip flips %s"
          % (i, Ho, Wo, y.shape[-1], int(fh.sum()), int(f32.sum()), float(a64.abs().min()),
             [float(v) for v in a64[fh].abs().cpu()[:5]]))
