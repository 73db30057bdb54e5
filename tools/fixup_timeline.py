"""Per-workgroup timeline of the split-K fix-up in the ConvT forward launches (damc_clock_probe stamps on X3_FIXUP
launches: K-loop end, slabs drained, wait over, bands done; 100 MHz realtime), CIFAR B=16 (run through gpurun)."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib, langevin as lv, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

os.environ["DAMC_X3_FIXUP"] = "1"  # the opt-in fix-up
dev = torch.device("cuda:0")
L = _lib.lib()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
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
c = c[c[:, 0] > 0]
t0 = c[:, 0].min()
q = torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0], dtype=torch.float64)
for i, name in enumerate(("K-loop end", "slabs drained", "wait over", "bands done")):
    print("%-14s us q0/10/50/90/100 %s" % (name, [round(float(v), 2) for v in torch.quantile((c[:, i] - t0) / 100.0, q)]))
print("drain (us) q", [round(float(v), 2) for v in torch.quantile((c[:, 1] - c[:, 0]) / 100.0, q)])
print("wait  (us) q", [round(float(v), 2) for v in torch.quantile((c[:, 2] - c[:, 1]) / 100.0, q)])
print("bands (us) q", [round(float(v), 2) for v in torch.quantile((c[:, 3] - c[:, 2]) / 100.0, q)])
