"""Localise GPU-vs-oracle differences at the BASELINE size (debug helper)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'diffusion-amortized-mcmc_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
import numpy as np, torch
from conftest import rel_l2
from test_gpu_langevin import _cifar_full
from damc import langevin as lv
from oracle import damc_oracle as orc
torch.set_num_threads(16)
dev = torch.device('cuda:0')
for B in (8, 16, 32, 64, 128):
    G, E, x, z0 = _cifar_full(dev, B)
    L, P = orc.generator_layers(G), orc.ebm_params(E)
    xh = lv.generator_forward(z0, G).cpu(); xr = orc.generator_sample(L, z0.cpu())
    g = lv.likelihood_grad(z0, x, G, 0.1).cpu(); gr, _, _ = orc.likelihood_grad(L, z0.cpu(), x.cpu(), 0.1)
    e, ge = lv.ebm_energy_grad(z0, E); er, ger = orc.ebm_energy_grad(P, z0.cpu())
    row = ((g - gr).norm(dim=1) / gr.norm(dim=1)).numpy()
    print(B, 'xhat %.2e' % rel_l2(xh.numpy(), xr.numpy()), 'glik %.2e' % rel_l2(g.numpy(), gr.numpy()),
          'gE %.2e' % rel_l2(ge.cpu().numpy(), ger.numpy()), 'worst rows', np.argsort(row)[-4:], row.max(), np.median(row))
    gr64, _, _ = orc.likelihood_grad(orc.generator_layers(G, torch.float64), z0.cpu().double(), x.cpu().double(), 0.1)
    print('   vs fp64: gpu %.2e  oracle32 %.2e' % (rel_l2(g.numpy(), gr64.numpy()), rel_l2(gr.numpy(), gr64.numpy())))
