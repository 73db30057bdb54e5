"""Q-update gradient errors vs the reference golden, per parameter: HIP drop-in on the GPU, stock PyTorch on the GPU
and stock PyTorch on the CPU (which config / which op departs).  usage: python tools/diag_qtrain.py q_celeba64_s"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from conftest import load_golden, qtrain_run  # noqa: E402

from damc import training  # noqa: E402


def errs(grads, rec, meta):
    out = []
    norms = [float(rec["grad%d_norm" % k]) for k in range(len(meta["params"]))]
    floor = 1e-3 * max(norms)
    for k, (pname, st, shape) in enumerate(meta["params"]):
        g = np.asarray(grads[k], dtype=np.float64).reshape(-1)
        ref = np.asarray(rec["grad%d_sub" % k], dtype=np.float64)
        den = max(np.linalg.norm(ref), floor * np.sqrt(ref.size / max(g.size, 1)), 1e-30)
        out.append((pname, float(np.linalg.norm(g[::st] - ref) / den)))
    return out


name = sys.argv[1] if len(sys.argv) > 1 else "q_celeba64_s"
dev = torch.device("cuda:0")
loss_h, g_h, rec, meta = qtrain_run(name, dev)
with training.stock_pytorch():
    loss_t, g_t, _, _ = qtrain_run(name, dev)
loss_c, g_c, _, _ = qtrain_run(name, "cpu")
eh, et, ec = errs(g_h, rec, meta), errs(g_t, rec, meta), errs(g_c, rec, meta)
print("loss rel err: hip %.2e torch-gpu %.2e cpu %.2e" % tuple(
    np.linalg.norm(l - rec["loss"]) / np.linalg.norm(rec["loss"]) for l in (loss_h, loss_t, loss_c)))
for (n, a), (_, b), (_, c) in zip(eh, et, ec):
    flag = " <==" if a > 3e-5 else ""
    print("%-40s hip %.2e  torch-gpu %.2e  cpu %.2e%s" % (n, a, b, c, flag))
