import os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch
from conftest import rel_l2
import test_gpu_configs as t
from damc import langevin as lv
from oracle import damc_oracle as orc
dev = torch.device("cuda:0")
for name, B in (("svhn", 64), ("celeba64", 256), ("celeba64", 32), ("svhn", 4)):
    G, E, x, z0 = t._case(name, B, dev)
    (L32, P32), (L64, P64) = t._oracles(G, E)
    g = lv.likelihood_grad(z0, x, G, 0.1).cpu().numpy()
    g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 0.1)[0].numpy()
    g32 = orc.likelihood_grad(L32, z0.cpu(), x.cpu(), 0.1)[0].numpy()
    e, ge = lv.ebm_energy_grad(z0, E)
    e64, ge64 = orc.ebm_energy_grad(P64, z0.cpu().double())
    xh = lv.generator_forward(z0, G).cpu().numpy()
    x64 = orc.generator_sample(L64, z0.cpu().double()).numpy()
    print(name, B, "lik grad %.2e (fp32 ref %.2e)  ebm e %.2e grad %.2e  G(z) %.2e" % (
        rel_l2(g, g64), rel_l2(g32, g64), rel_l2(e.cpu().numpy(), e64.numpy()), rel_l2(ge.cpu().numpy(), ge64.numpy()),
        rel_l2(xh, x64)))
from damc import _lib
with _lib.exact_fp32():
    for name, B in (("svhn", 64), ("celeba64", 256)):
        G, E, x, z0 = t._case(name, B, dev)
        (L32, P32), (L64, P64) = t._oracles(G, E)
        g = lv.likelihood_grad(z0, x, G, 0.1).cpu().numpy()
        g64 = orc.likelihood_grad(L64, z0.cpu().double(), x.cpu().double(), 0.1)[0].numpy()
        print("exact fp32 engine:", name, B, "lik grad %.2e" % rel_l2(g, g64))
# repeatability: same call twice
G, E, x, z0 = t._case("svhn", 64, dev)
a = lv.likelihood_grad(z0, x, G, 0.1).cpu()
b = lv.likelihood_grad(z0, x, G, 0.1).cpu()
print("repeat identical:", torch.equal(a, b), "max diff %.3e" % (a - b).abs().max().item())
# per-row error: which samples are off
g64 = orc.likelihood_grad(t._oracles(G, E)[1][0], z0.cpu().double(), x.cpu().double(), 0.1)[0]
err = ((a.double() - g64).norm(dim=1) / g64.norm(dim=1)).numpy()
print("per-row rel err:", " ".join("%.0e" % v for v in err))
