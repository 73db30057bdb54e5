"""Toy configuration #1 (workspace/toy_example/toy_example.py): 2-D latent, MLP likelihood G.

``ToyG`` has the reference's module layout (``net`` = Linear(2,128) ReLU Linear(128,128) ReLU
Linear(128,128) ReLU Linear(128,2), toy_example.py:22-47) so its state_dict matches; weights are
loaded by the caller.  ``posterior`` runs the toy's Langevin closure (toy_example.py:110-131:
U = |G(z)-x|^2/(2*.25^2) + |z|^2/2, no EBM) on the HIP path.
"""
import torch
import torch.nn as nn


class ToyG(nn.Module):
    def __init__(self, nz=2, width=128):
        super().__init__()
        dims = [nz, width, width, width, nz]
        mods = []
        for i, (a, b) in enumerate(zip(dims[:-1], dims[1:])):
            mods.append(nn.Linear(a, b))
            if i < len(dims) - 2:
                mods.append(nn.ReLU())
        self.net = nn.Sequential(*mods)

    def forward(self, z):
        return self.net(z)


def posterior(z, x, G, n_steps, step=0.1, sigma=0.25, with_noise=True, noise=None, seed=None):
    from . import langevin

    return langevin.posterior_langevin(z, x, G, None, n_steps, sigma, step, with_noise, noise=noise, seed=seed)
