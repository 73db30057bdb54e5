"""Workgroup start / K-loop end spread of one limb-engine ConvT forward launch (damc_clock_probe stamps, 100 MHz
realtime): is the split-K grid co-resident, and how far apart do its workgroups finish?  (run through gpurun)"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib, langevin as lv, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

dev = torch.device("cuda:0")
L = _lib.lib()
for fix in ("1", "0"):
    os.environ["DAMC_X3_FIXUP"] = fix
    for B in (16, 128):
        G = synth.load_into(dn._netG_cifar10(nz=128, ngf=128, nc=3), 0).to(dev).eval()
        E = synth.load_into(dn._netE(nz=128), 10).to(dev).eval()
        x = torch.from_numpy(synth.uniform_f32(61, 0, (B, 3, 32, 32))).to(dev)
        z = torch.from_numpy(synth.normal_f32(62, 0, (B, 128))).to(dev)
        lv.posterior_langevin(z, x, G, E, 2, 0.1, 0.1, True, seed=9)
        clk = torch.zeros(1024 * 4, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        L.damc_clock_probe(clk.data_ptr(), 1024)
        lv.posterior_langevin(z, x, G, E, 1, 0.1, 0.1, True, seed=9)
        torch.cuda.synchronize()
        L.damc_clock_probe(None, 0)
        c = clk.view(-1, 4).cpu().double()
        c = c[c[:, 1] > 0]
        t0 = c[:, 1].min()
        st, en = (c[:, 1] - t0) / 100.0, (c[:, 3] - t0) / 100.0
        q = torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0], dtype=torch.float64)
        print("FIXUP=%s B=%d: %d workgroups; start us q0/10/50/90/100 %s; K-loop end %s" % (
            fix, B, len(c), [round(float(v), 1) for v in torch.quantile(st, q)],
            [round(float(v), 1) for v in torch.quantile(en, q)]), flush=True)
