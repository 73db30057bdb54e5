# where the CelebA-HQ likelihood-gradient error comes from: forward G(z) per row, and tiny generators that isolate
# the proj layer's dgrad (K = 16 C) and the k4 s2 output layer, each vs fp64 and the CPU fp32 oracle
import os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE, os.path.join(HERE, "tools")]
import numpy as np
import torch
from conftest import rel_l2
from damc import synth, langevin as lv
from oracle import damc_oracle as orc
import test_gpu_configs as t
dev = torch.device("cuda:0")
rows = lambda a, r: np.array([rel_l2(a[i], r[i]) for i in range(r.shape[0])])

G, E, x, z0 = t._case("celebaHQ", 8, dev)
(L32, _), (L64, _) = t._oracles(G, E)
xh = lv.generator_forward(z0, G).cpu().numpy()
x64 = orc.generator_sample(L64, z0.cpu().double()).numpy()
x32 = orc.generator_sample(L32, z0.cpu()).numpy()
print("HQ G(z) per-row median hip %.2e cpu %.2e" % (np.median(rows(xh, x64)), np.median(rows(x32, x64))), flush=True)

class Gen(torch.nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.gen = torch.nn.Sequential(*layers)

def make(nz, C, up, Cl):
    L = [torch.nn.ConvTranspose2d(nz, C, 4, 1, 0), torch.nn.LeakyReLU(0.2)]
    c = C
    for _ in range(up):
        L += [torch.nn.ConvTranspose2d(c, c // 2, 4, 2, 1), torch.nn.LeakyReLU(0.2)]
        c //= 2
    L += [torch.nn.ConvTranspose2d(c, Cl, 4, 2, 1), torch.nn.Tanh()]
    return synth.load_into(Gen(L), 0).to(dev).eval()

for nz, C, up, Cl, B in ((128, 256, 0, 3, 8), (128, 512, 0, 3, 8), (128, 2048, 0, 3, 8), (128, 1024, 2, 3, 8),
                         (128, 2048, 3, 3, 8), (128, 2048, 3, 3, 32)):
    G = make(nz, C, up, Cl)
    hw = 4 * 2 ** (up + 1)
    x = torch.rand(B, Cl, hw, hw, device=dev) * 2 - 1
    z = torch.randn(B, nz, device=dev)
    L32, L64 = orc.generator_layers(G), orc.generator_layers(G, torch.float64)
    try:
        g = lv.likelihood_grad(z, x, G, 1.0).cpu().numpy()
    except Exception as e:
        print(nz, C, up, Cl, B, "unsupported:", e)
        continue
    g64 = orc.likelihood_grad(L64, z.cpu().double(), x.cpu().double(), 1.0)[0].numpy()
    g32 = orc.likelihood_grad(L32, z.cpu(), x.cpu(), 1.0)[0].numpy()
    print("proj %d->%d, %d up, out %d, B=%d: lik grad per-row median hip %.2e cpu %.2e" % (
        nz, C, up, Cl, B, np.median(rows(g, g64)), np.median(rows(g32, g64))), flush=True)
