import os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch
import test_gpu_configs as t
from damc import langevin as lv
from oracle import damc_oracle as orc
dev = torch.device("cuda:0")
G, E, x, z0 = t._case("svhn", 64, dev)
(L32, P32), (L64, P64) = t._oracles(G, E)
g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 0.1)[0]
def rowerr(g, rows):
    return ((g.cpu().double() - g64[rows]).norm(dim=1) / g64[rows].norm(dim=1)).numpy()
full = lv.likelihood_grad(z0, x, G, 0.1)
e = rowerr(full, slice(0, 64))
bad = [i for i in range(64) if e[i] > 1e-4]
print("bad rows in B=64:", bad, ["%.1e" % e[i] for i in bad])
for lo, hi in ((54, 55), (48, 64), (32, 64), (0, 55), (0, 56), (40, 60), (50, 58)):
    g = lv.likelihood_grad(z0[lo:hi].contiguous(), x[lo:hi].contiguous(), G, 0.1)
    e = rowerr(g, slice(lo, hi))
    print("B=%d rows [%d,%d): bad" % (hi - lo, lo, hi), [lo + i for i in range(hi - lo) if e[i] > 1e-4], "max %.1e" % e.max())
# x-only: swap row 54's x with row 0's
zz = z0.clone(); xx = x.clone(); zz[54] = z0[0]
g = lv.likelihood_grad(zz, xx, G, 0.1)
g64b = orc.likelihood_grad(L64, zz.cpu().double(), xx.cpu().double(), 0.1)[0]
eb = ((g.cpu().double() - g64b).norm(dim=1) / g64b.norm(dim=1)).numpy()
print("row 54 <- z of row 0: bad", [i for i in range(64) if eb[i] > 1e-4])
