#!/usr/bin/env python
"""Capture golden vectors from the REFERENCE implementation (build container only).

This script imports the reference's own modules from /root/reference (read-only)
and records their outputs on counter-hash inputs (damc.synth) into small .npz
fixtures under tests/golden/.  It is never run on the GPU box and nothing in
tests/, bench.py or __graft_entry__ imports it; the tests only read the .npz.

Reference entry points exercised (all unchanged):
  * sample_langevin_post_z_with_prior   workspace/src/MCMC.py:48-74
  * sample_langevin_prior_z             workspace/src/MCMC.py:27-46
  * _netG_* forward                     workspace/src/diffusion_net.py:20-203
  * _netE forward                       workspace/src/diffusion_net.py:207-223
  * Encoder_* forward                   workspace/src/diffusion_net.py:227-413
  * _netQ_U.forward (reverse sweep)     workspace/src/diffusion_net.py:585-622
  * toy G + the toy's posterior update  workspace/toy_example/toy_example.py:22-47,110-131
    (the toy closure is the a1 update with E == 0 and sigma = .25; it is driven
    here through the reference's sample_langevin_post_z_with_prior with a zero
    energy net, which performs the identical arithmetic)

Noise injection: torch.randn / torch.randn_like are patched to return the next
counter-hash array (damc.synth.normal_f32) so our build can be fed exactly the
same noise through its injected-noise buffer.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import json
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "diffusion-amortized-mcmc_amd"))
REF_WS = "/root/reference/workspace"

from damc import synth  # noqa: E402

# our drop-in package is also called `src` (a regular package), and the reference's `src` is a
# namespace package, which the import system would skip in favour of ours: drop our path now.
sys.path.pop(0)

# ---- seeds / streams shared with tests (tests/golden/README in conftest) ----
SEED_G, SEED_E, SEED_Q = 0, 10, 20
SEED_X, SEED_Z0, SEED_POST, SEED_PRIOR, SEED_PRIOR_INIT, SEED_QN = 1, 2, 3, 4, 5, 6

G_CONFIGS = {
    # name: (ctor, nz, ngf, nc, H, B)
    "svhn_w16": ("_netG_svhn", 100, 16, 3, 32, 4),
    "cifar10_w16": ("_netG_cifar10", 128, 16, 3, 32, 4),
    "celeba64_w16": ("_netG_celeba64", 100, 16, 3, 64, 3),
    "celebaHQ_w8": ("_netG_celebaHQ", 128, 8, 3, 256, 2),
    "mnist_w16": ("_netG_mnist", 100, 16, 1, 28, 4),
    "cifar10_full": ("_netG_cifar10", 128, 128, 3, 32, 8),
}

Q_CONFIGS = {
    # name: (dataset, nc, nz, nif, nxemb, ntemb, H, B, var_type, n_interval)
    "q_cifar10_s": ("cifar10", 3, 128, 8, 64, 32, 32, 4, "large", 100),
    "q_cifar10_small": ("cifar10", 3, 128, 8, 64, 32, 32, 4, "small", 12),
    "q_svhn_s": ("svhn", 3, 100, 8, 64, 32, 32, 3, "large", 100),
    "q_celeba64_s": ("celeba64", 3, 100, 8, 64, 32, 64, 2, "large", 20),
    "q_celebaHQ_s": ("celebaHQ", 3, 128, 4, 64, 32, 256, 2, "large", 10),
    "q_mnist_s": ("mnist", 1, 100, 8, 64, 32, 28, 3, "large", 20),
    "q_cifar10_full": ("cifar10", 3, 128, 64, 1024, 128, 32, 4, "large", 100),
}


class NoiseQueue:
    def __init__(self):
        self.items = []

    def push(self, arr):
        self.items.append(arr)

    def pop(self, shape):
        arr = self.items.pop(0)
        assert tuple(arr.shape) == tuple(shape), (arr.shape, shape)
        return arr


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    # MCMC.py imports torchvision / pytorch_fid_wrapper at top level but only uses
    # them in the FID/image helpers (workspace/src/MCMC.py:7-8,139-142).
    for name in ("torchvision", "torchvision.utils", "pytorch_fid_wrapper"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.path.insert(0, REF_WS)
    import src.diffusion_net as dn  # noqa
    import src.MCMC as mc  # noqa
    return dn, mc


def patch_randn(torch, q):
    orig_randn, orig_randn_like = torch.randn, torch.randn_like

    def fake_randn(*size, **kw):
        if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)):
            size = tuple(size[0])
        arr = q.pop(tuple(size))
        return torch.from_numpy(arr.copy()).to(kw.get("device") or "cpu")

    def fake_randn_like(t, **kw):
        arr = q.pop(tuple(t.shape))
        return torch.from_numpy(arr.copy()).to(t.device)

    torch.randn, torch.randn_like = fake_randn, fake_randn_like
    return orig_randn, orig_randn_like


def capture_generators(dn, mc, torch):
    out = {}
    for name, (ctor, nz, ngf, nc, H, B) in G_CONFIGS.items():
        print("G config", name, flush=True)
        G = getattr(dn, ctor)(nz=nz, ngf=ngf, nc=nc)
        E = dn._netE(nz=nz)
        synth.load_into(G, SEED_G)
        synth.load_into(E, SEED_E)
        G.eval(), E.eval()
        x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H)))
        z0 = torch.from_numpy(synth.normal_f32(SEED_Z0, 0, (B, nz)))
        rec = {}
        sigma, s = 0.1, 0.1
        with torch.no_grad():
            gx = G(z0).numpy()
            if H > 64:      # keep the fixture small: every 4th pixel of the 256^2 image
                rec["gen_x_sub4"] = gx[:, :, ::4, ::4].copy()
            else:
                rec["gen_x"] = gx
            rec["ebm_e"] = E(z0).numpy()
        # exact gradients of the three energy terms at z0 (the terms of workspace/src/MCMC.py:56-60)
        z = z0.clone().requires_grad_(True)
        lik = 1.0 / (2.0 * sigma * sigma) * torch.sum((G(z) - x) ** 2)
        rec["lik_grad0"] = torch.autograd.grad(lik, z)[0].numpy()
        z = z0.clone().requires_grad_(True)
        rec["ebm_grad0"] = torch.autograd.grad(E(z).sum(), z)[0].numpy()
        rec["lik0"] = np.float32(lik.item())
        # 1 step, no noise -> gradient of U at z0
        z = z0.clone().requires_grad_(True)
        z1 = mc.sample_langevin_post_z_with_prior(z, x, G, E, 1, sigma, False, s)
        rec["post_z1"] = z1.numpy().copy()
        # 10 steps, no noise (eval path, workspace/eval_gen_recon.py:184-194)
        z = z0.clone().requires_grad_(True)
        z10 = mc.sample_langevin_post_z_with_prior(z, x, G, E, 10, sigma, False, s)
        rec["post_z10"] = z10.numpy().copy()
        with torch.no_grad():
            rec["recon_mse10"] = torch.mean((G(z10) - x) ** 2, dim=[1, 2, 3]).numpy()
        # 30 steps with injected noise (train path, workspace/train_gen_recon.py:203-205)
        q = NoiseQueue()
        for i in range(30):
            q.push(synth.normal_f32(SEED_POST, 100 + i, (B, nz)))
        saved = patch_randn(torch, q)
        try:
            z = z0.clone().requires_grad_(True)
            z30 = mc.sample_langevin_post_z_with_prior(z, x, G, E, 30, sigma, True, s)
        finally:
            torch.randn, torch.randn_like = saved
        rec["post_z30"] = z30.numpy().copy()
        # prior: 60 steps on 2B chains, s=.4 (workspace/train_gen_recon.py:206-209)
        zp0 = np.concatenate([z0.numpy(), synth.normal_f32(SEED_PRIOR_INIT, 0, (B, nz))], 0)
        q = NoiseQueue()
        for i in range(60):
            q.push(synth.normal_f32(SEED_PRIOR, 100 + i, (2 * B, nz)))
        saved = patch_randn(torch, q)
        try:
            z = torch.from_numpy(zp0.copy()).requires_grad_(True)
            zp = mc.sample_langevin_prior_z(z, E, 60, 0.4, True)
        finally:
            torch.randn, torch.randn_like = saved
        rec["prior_z60"] = zp.numpy().copy()
        # prior 5 steps no noise (tight per-step tolerance)
        z = torch.from_numpy(zp0.copy()).requires_grad_(True)
        rec["prior_z5"] = mc.sample_langevin_prior_z(z, E, 5, 0.4, False).numpy().copy()
        meta = dict(kind="G", ctor=ctor, nz=nz, ngf=ngf, nc=nc, H=H, B=B, sigma=sigma, step=s,
                    prior_step=0.4, g_keys=[[k, list(v.shape)] for k, v in G.state_dict().items()],
                    e_keys=[[k, list(v.shape)] for k, v in E.state_dict().items()])
        out[name] = (rec, meta)
    return out


def capture_gtrain(dn, torch):
    """The G update (workspace/train_gen_recon.py:222-231) on the reference generator: x_hat = G(z0),
    g_loss = sum((x_hat - x)^2, [1,2,3]).mean(), g_loss.backward().  Every parameter gradient is kept as
    an evenly strided subsample (<= 2048 values) plus its full L2 norm, to keep the fixtures small."""
    out = {}
    for name, (ctor, nz, ngf, nc, H, B) in G_CONFIGS.items():
        print("G train config", name, flush=True)
        G = getattr(dn, ctor)(nz=nz, ngf=ngf, nc=nc)
        synth.load_into(G, SEED_G)
        G.train()
        x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H)))
        z0 = torch.from_numpy(synth.normal_f32(SEED_Z0, 0, (B, nz)))
        G.zero_grad()
        x_hat = G(z0)
        g_loss = torch.sum((x_hat - x) ** 2, dim=[1, 2, 3]).mean()
        g_loss.backward()
        rec = {"g_loss": np.float32(g_loss.item())}
        strides = []
        for k, (pname, p) in enumerate(G.named_parameters()):
            g = p.grad.detach().numpy().reshape(-1)
            st = max(1, g.size // 2048)
            rec["grad%d_sub" % k] = g[::st].copy()
            rec["grad%d_norm" % k] = np.float64(np.linalg.norm(g.astype(np.float64)))
            strides.append([pname, st, list(p.shape)])
        meta = dict(kind="Gtrain", ctor=ctor, nz=nz, ngf=ngf, nc=nc, H=H, B=B, params=strides)
        out[name + "_gtrain"] = (rec, meta)
    return out


def capture_checkpoint(dn, torch):
    """A training checkpoint in the reference's format (workspace/train_gen_recon.py:284-294), written by the
    reference's own modules and optimizers after one G / Q / E update at tiny widths, plus the reference G's
    output on fixed inputs after loading it (tests/test_oracle_golden.py::test_reference_checkpoint_loads)."""
    import torch.optim as optim

    nz = 16
    G = dn._netG_cifar10(nz=nz, ngf=4, nc=3)
    E = dn._netE(nz=nz, ndf=8)
    qargs = dict(nc=3, nz=nz, nxemb=16, ntemb=16, nf=1, nif=2, diffusion_residual=True, n_interval=4,
                 logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                 dataset="cifar10")
    Q, Q_dummy = dn._netQ_U(**qargs), dn._netQ_U(**qargs)
    for i, m in enumerate((G, E, Q, Q_dummy)):
        synth.load_into(m, 50 + i)
    G_opt = optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
    Q_opt = optim.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
    E_opt = optim.Adam(E.parameters(), lr=1e-4, betas=(0.5, 0.999))
    x = torch.from_numpy(synth.uniform_f32(60, 0, (4, 3, 32, 32)))
    z = torch.from_numpy(synth.normal_f32(61, 0, (4, nz)))
    torch.manual_seed(0)
    G_opt.zero_grad()
    torch.sum((G(z) - x) ** 2, dim=[1, 2, 3]).mean().backward()
    G_opt.step()
    Q_opt.zero_grad()
    Q.calculate_loss(x=x, z=z, mask=torch.ones(4, 1)).mean().backward()
    Q_opt.step()
    E_opt.zero_grad()
    (E(z).mean() - E(-z).mean()).backward()
    E_opt.step()
    save_dict = {"G_state_dict": G.state_dict(), "G_optimizer": G_opt.state_dict(), "Q_state_dict": Q.state_dict(),
                 "Q_optimizer": Q_opt.state_dict(), "Q_dummy_state_dict": Q_dummy.state_dict(),
                 "E_state_dict": E.state_dict(), "E_optimizer": E_opt.state_dict(), "iter": 1}
    torch.save(save_dict, os.path.join(HERE, "ckpt_cifar10_tiny.pth.tar"))
    with torch.no_grad():
        rec = {"gen_x": G(z).numpy(), "ebm_e": E(z).numpy(), "xemb": Q.encoder(x).numpy()}
    meta = dict(kind="ckpt", nz=nz, ngf=4, ndf=8, q=qargs)
    np.savez(os.path.join(HERE, "ckpt_cifar10_tiny.npz"), meta=json.dumps(meta), **rec)


QTRAIN_CONFIGS = ["q_cifar10_s", "q_svhn_s", "q_mnist_s", "q_cifar10_full", "q_celeba64_s", "q_celebaHQ_s"]
SEED_QT = 7


def qtrain_noise(B, nz):
    """The random draws of one Q.calculate_loss call (diffusion_net.py:624-641), in call order:
    prior_emb input randn(B, nz), u = rand(B), eps = randn_like(z)."""
    return (synth.normal_f32(SEED_QT, 0, (B, nz)), synth.uniform_f32(SEED_QT, 1, (B,), 0.0, 1.0),
            synth.normal_f32(SEED_QT, 2, (B, nz)))


def capture_qtrain(dn, torch):
    """The Q update's loss (workspace/train_gen_recon.py:211-217): Q.train(); Q.calculate_loss(x, z,
    mask).mean().backward() on the reference Q with injected noise and a mixed mask; per-sample losses and
    every parameter gradient (strided subsample <= 512 values + full L2 norm)."""
    out = {}
    for name in QTRAIN_CONFIGS:
        ds, nc, nz, nif, nxemb, ntemb, H, B, var_type, n_int = Q_CONFIGS[name]
        print("Q train config", name, flush=True)
        Q = dn._netQ_U(nc=nc, nz=nz, nxemb=nxemb, ntemb=ntemb, nif=nif, diffusion_residual=True,
                       n_interval=n_int, logsnr_min=-5.1, logsnr_max=9.8, var_type=var_type,
                       with_noise=True, cond_w=0.0, net_arch="A", dataset=ds)
        synth.load_into(Q, SEED_Q)
        Q.train()
        x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H)))
        z = torch.from_numpy(synth.normal_f32(SEED_Z0, 0, (B, nz)))
        mask = torch.ones(B, 1)
        mask[1::3] = 0.0
        pe, u, eps = qtrain_noise(B, nz)
        orig = torch.randn, torch.rand, torch.randn_like
        torch.randn = lambda *a, **k: torch.from_numpy(pe.copy())
        torch.rand = lambda *a, **k: torch.from_numpy(u.copy())
        torch.randn_like = lambda t, **k: torch.from_numpy(eps.copy())
        try:
            Q.zero_grad()
            loss = Q.calculate_loss(x=x, z=z, mask=mask)
            loss.mean().backward()
        finally:
            torch.randn, torch.rand, torch.randn_like = orig
        rec = {"loss": loss.detach().numpy()}
        params = []
        for k, (pname, p) in enumerate(Q.named_parameters()):
            if p.grad is None:
                continue
            g = p.grad.detach().numpy().reshape(-1)
            st = max(1, g.size // 512)
            rec["grad%d_sub" % len(params)] = g[::st].copy()
            rec["grad%d_norm" % len(params)] = np.float64(np.linalg.norm(g.astype(np.float64)))
            params.append([pname, st, list(p.shape)])
        meta = dict(kind="Qtrain", q=name, params=params)
        out[name + "_qtrain"] = (rec, meta)
    return out


def capture_q(dn, torch):
    out = {}
    for name, (ds, nc, nz, nif, nxemb, ntemb, H, B, var_type, n_int) in Q_CONFIGS.items():
        print("Q config", name, flush=True)
        Q = dn._netQ_U(nc=nc, nz=nz, nxemb=nxemb, ntemb=ntemb, nif=nif, diffusion_residual=True,
                       n_interval=n_int, logsnr_min=-5.1, logsnr_max=9.8, var_type=var_type,
                       with_noise=True, cond_w=0.0, net_arch="A", dataset=ds)
        synth.load_into(Q, SEED_Q)
        Q.eval()
        x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H)))
        rec = {}
        eps_log = []
        h = Q.p.register_forward_hook(lambda m, i, o: eps_log.append(o.detach().numpy().copy()))
        with torch.no_grad():
            rec["xemb"] = Q.encoder(x).numpy()
            # posterior sweep Q(x): randn for zt, then randn_like per step i>0
            q = NoiseQueue()
            q.push(synth.normal_f32(SEED_QN, 0, (B, nz)))
            for i in range(n_int - 1):
                q.push(synth.normal_f32(SEED_QN, 100 + i, (B, nz)))
            saved = patch_randn(torch, q)
            try:
                rec["q_post"] = Q(x).numpy()
            finally:
                torch.randn, torch.randn_like = saved
            rec["q_post_eps3"] = np.stack(eps_log[:3])
            eps_log.clear()
            # prior sweep Q(x=None, b): randn for prior_emb input, randn for zt, eps per step
            q = NoiseQueue()
            q.push(synth.normal_f32(SEED_QN, 1, (B, nz)))
            q.push(synth.normal_f32(SEED_QN, 0, (B, nz)))
            for i in range(n_int - 1):
                q.push(synth.normal_f32(SEED_QN, 100 + i, (B, nz)))
            saved = patch_randn(torch, q)
            try:
                rec["q_prior"] = Q(x=None, b=B, device=torch.device("cpu")).numpy()
            finally:
                torch.randn, torch.randn_like = saved
            rec["q_prior_eps3"] = np.stack(eps_log[:3])
        h.remove()
        meta = dict(kind="Q", dataset=ds, nc=nc, nz=nz, nif=nif, nxemb=nxemb, ntemb=ntemb, H=H, B=B,
                    var_type=var_type, n_interval=n_int, logsnr_min=-5.1, logsnr_max=9.8,
                    q_keys=[[k, list(v.shape)] for k, v in Q.state_dict().items()])
        out[name] = (rec, meta)
    return out


TOY_CHILD = r"""
import sys, types, os, json
import numpy as np
sys.dont_write_bytecode = True
repo, ws, out = sys.argv[1], sys.argv[2], sys.argv[3]
sys.path.insert(0, os.path.join(repo, 'diffusion-amortized-mcmc_amd'))
for n in ('matplotlib', 'matplotlib.pyplot'):
    sys.modules.setdefault(n, types.ModuleType(n))
sys.path.insert(0, os.path.join(ws, 'toy_example'))
import torch
torch.set_num_threads(8)
from damc import synth
sys.path.pop(1)
import toy_example                      # workspace/toy_example/toy_example.py (class G)
G = toy_example.G()
synth.load_into(G, 0)
B, nz, steps, s, sigma = 500, 2, 1000, 0.1, 0.25
zstar = torch.from_numpy(synth.normal_f32(1, 0, (B, nz)))
with torch.no_grad():
    x = G(zstar) + 0.25 * torch.from_numpy(synth.normal_f32(1, 1, (B, nz)))
z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, nz)))
noise = [synth.normal_f32(3, 100 + i, (B, nz)) for i in range(steps)]
# workspace/src as package `wsrc` (the toy tree already owns the name `src`)
for n in ('torchvision', 'torchvision.utils', 'pytorch_fid_wrapper'):
    sys.modules.setdefault(n, types.ModuleType(n))
pkg = types.ModuleType('wsrc'); pkg.__path__ = [os.path.join(ws, 'src')]; sys.modules['wsrc'] = pkg
import importlib
mc = importlib.import_module('wsrc.MCMC')
class ZeroE(torch.nn.Module):          # the toy closure has no EBM term (toy_example.py:117-119)
    def forward(self, z):
        return torch.zeros(len(z))
it = iter(noise)
torch.randn_like = lambda t, **kw: torch.from_numpy(next(it).copy())
z = z0.clone().requires_grad_(True)
z1 = mc.sample_langevin_post_z_with_prior(z, x, G, ZeroE(), 1, sigma, True, s).numpy().copy()
it = iter(noise)
z = z0.clone().requires_grad_(True)
zN = mc.sample_langevin_post_z_with_prior(z, x, G, ZeroE(), steps, sigma, True, s).numpy().copy()
np.savez(out, x=x.numpy(), post_z1=z1, post_z1000=zN,
         meta=json.dumps(dict(kind='toy', B=B, nz=nz, steps=steps, step=s, sigma=sigma)))
"""


def main():
    import torch

    torch.set_num_threads(8)
    dn, mc = import_reference()
    if "--qtrain-only" not in sys.argv:
        capture_checkpoint(dn, torch)
    for name, (rec, meta) in capture_qtrain(dn, torch).items():
        np.savez(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **rec)
    if "--qtrain-only" in sys.argv:
        print("done")
        return
    for name, (rec, meta) in capture_gtrain(dn, torch).items():
        np.savez(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **rec)
    if "--gtrain-only" in sys.argv:
        print("done")
        return
    for name, (rec, meta) in capture_generators(dn, mc, torch).items():
        np.savez(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **rec)
    for name, (rec, meta) in capture_q(dn, torch).items():
        np.savez(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **rec)
    # toy in its own process: both reference trees name their package `src`
    subprocess.check_call([sys.executable, "-c", TOY_CHILD, REPO, REF_WS,
                           os.path.join(HERE, "toy.npz")],
                          env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    print("done")


if __name__ == "__main__":
    main()
