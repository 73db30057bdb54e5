"""pytest configuration.

Markers: ``gpu`` — needs a ROCm device and libdamc.so (run on the MI355X box with -m gpu).

Golden fixtures (tests/golden/*.npz) were captured from the REFERENCE implementation by
tests/golden/make_golden.py (build container only).  Inputs are regenerated here from the
counter-hash recipe (damc.synth) with the seeds below, which the capture script used too.
"""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "diffusion-amortized-mcmc_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# seeds shared with tests/golden/make_golden.py
SEED_G, SEED_E, SEED_Q = 0, 10, 20
SEED_X, SEED_Z0, SEED_POST, SEED_PRIOR, SEED_PRIOR_INIT, SEED_QN = 1, 2, 3, 4, 5, 6

G_NAMES = ["svhn_w16", "cifar10_w16", "celeba64_w16", "celebaHQ_w8", "mnist_w16", "cifar10_full"]
Q_NAMES = ["q_cifar10_s", "q_cifar10_small", "q_svhn_s", "q_celeba64_s", "q_celebaHQ_s", "q_mnist_s",
           "q_cifar10_full"]
# End-point backstop (rel-L2 from the reference golden) of a full reverse sweep; the real criterion is accuracy-relative
# (|hip - fp64| <= 3 |reference - fp64|, tests/test_gpu_amortizer.py).  n_interval 10-20 sweeps amplify rounding through
# sqrt(1+e^-l) every step, so the reference's own fp32 result sits 3e-4 .. 8e-2 from an fp64 evaluation of the same
# sweep (|reference - fp64|, per case).  Bound: 1.5x the largest |hip - reference| measured over the posterior and
# prior sweeps of two rounds' GPU runs (profiles/r02/sweep_end_distances.txt, profiles/r03/sweep_end_distances.txt),
# rounded up (q_cifar10_s keeps round 2's tighter 2e-2: measured 1.64e-2).  q_cifar10_full: 1.5x round 4's largest
# |hip - reference| over four GPU runs (8.0e-3; gpurun_out r4a/r4d/r4e logs).
Q_END_TOL = {"q_cifar10_s": 2e-2, "q_cifar10_small": 1.35e-1, "q_svhn_s": 1.1e-3, "q_celeba64_s": 1.0e-1,
             "q_celebaHQ_s": 9e-2, "q_mnist_s": 9e-2, "q_cifar10_full": 1.25e-2}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) device and libdamc.so")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.loads(str(d["meta"]))
    return {k: d[k] for k in d.files if k != "meta"}, meta


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def build_g_case(name, device="cpu"):
    """Nets + inputs of a golden generator case (drop-in classes, counter-hash weights)."""
    import torch

    from damc import synth
    from src import diffusion_net as dn

    rec, meta = load_golden(name)
    G = getattr(dn, meta["ctor"])(nz=meta["nz"], ngf=meta["ngf"], nc=meta["nc"])
    E = dn._netE(nz=meta["nz"])
    synth.load_into(G, SEED_G)
    synth.load_into(E, SEED_E)
    G.to(device).eval()
    E.to(device).eval()
    B, nz, nc, H = meta["B"], meta["nz"], meta["nc"], meta["H"]
    x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H))).to(device)
    z0 = torch.from_numpy(synth.normal_f32(SEED_Z0, 0, (B, nz))).to(device)
    post_noise = torch.from_numpy(np.stack([synth.normal_f32(SEED_POST, 100 + i, (B, nz)) for i in range(30)]))
    zp0 = torch.from_numpy(np.concatenate([z0.cpu().numpy(), synth.normal_f32(SEED_PRIOR_INIT, 0, (B, nz))], 0))
    prior_noise = torch.from_numpy(np.stack([synth.normal_f32(SEED_PRIOR, 100 + i, (2 * B, nz)) for i in range(60)]))
    return dict(G=G, E=E, x=x, z0=z0, post_noise=post_noise.to(device), zp0=zp0.to(device),
                prior_noise=prior_noise.to(device), rec=rec, meta=meta)


def gtrain_inputs(name):
    """G-update case (tests/golden/<name>_gtrain.npz): drop-in G with counter-hash weights, z0, x and
    dL/dx_hat of g_loss = sum((x_hat - x)^2, [1,2,3]).mean() (workspace/train_gen_recon.py:227-228)."""
    import torch

    from damc import synth
    from src import diffusion_net as dn

    rec, meta = load_golden(name + "_gtrain")
    G = getattr(dn, meta["ctor"])(nz=meta["nz"], ngf=meta["ngf"], nc=meta["nc"])
    synth.load_into(G, SEED_G)
    B, nz, nc, H = meta["B"], meta["nz"], meta["nc"], meta["H"]
    x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H)))
    z0 = torch.from_numpy(synth.normal_f32(SEED_Z0, 0, (B, nz)))
    return G, z0, x, rec, meta


def gtrain_errors(grads, rec, meta):
    """Per-parameter (subsample error, norm error) against the golden, as gtrain_check measures them."""
    out = []
    norms = [float(rec["grad%d_norm" % k]) for k in range(len(meta["params"]))]
    floor = 1e-3 * max(norms)
    for k, (pname, st, shape) in enumerate(meta["params"]):
        g = np.asarray(grads[k], dtype=np.float64).reshape(-1)
        ref = np.asarray(rec["grad%d_sub" % k], dtype=np.float64)
        den = max(np.linalg.norm(ref), floor * np.sqrt(ref.size / max(g.size, 1)), 1e-30)
        out.append((float(np.linalg.norm(g[::st] - ref) / den),
                    float(abs(np.linalg.norm(g) - norms[k]) / max(norms[k], floor, 1e-30))))
    return out


def gtrain_check(grads, rec, meta, tol):
    """Compare a list of per-parameter gradients (module order) with the golden subsamples/norms.

    Errors are relative to the tensor's own norm, floored at 1e-3 x the largest gradient norm of the net:
    a gradient that is analytically zero (e.g. the bias of a conv followed by InstanceNorm, whose mean the
    norm removes) is rounding noise in every implementation and is checked against that floor."""
    worst = 0.0
    norms = [float(rec["grad%d_norm" % k]) for k in range(len(meta["params"]))]
    floor = 1e-3 * max(norms)
    for k, (pname, st, shape) in enumerate(meta["params"]):
        g = np.asarray(grads[k], dtype=np.float64).reshape(-1)
        assert list(np.asarray(grads[k]).shape) == shape, (pname, np.asarray(grads[k]).shape, shape)
        ref = np.asarray(rec["grad%d_sub" % k], dtype=np.float64)
        den = max(np.linalg.norm(ref), floor * np.sqrt(ref.size / max(g.size, 1)), 1e-30)
        e = float(np.linalg.norm(g[::st] - ref) / den)
        n = abs(np.linalg.norm(g) - norms[k]) / max(norms[k], floor, 1e-30)
        worst = max(worst, e, n)
        t = tol[k] if isinstance(tol, (list, tuple)) else tol
        assert e < t and n < t, (pname, e, n, t)
    return worst


SEED_QT = 7  # tests/golden/make_golden.py qtrain_noise


def qtrain_run(name, device):
    """One Q.calculate_loss(x, z, mask).mean().backward() (train_gen_recon.py:211-217) of the drop-in Q with the
    golden case's injected noise; returns (per-sample loss, [grads in named_parameters order, grad != None],
    rec, meta)."""
    import torch

    from damc import synth
    from src import diffusion_net as dn

    rec, meta = load_golden(name + "_qtrain")
    c = build_q_case(meta["q"], device)
    Q, x, m = c["Q"], c["x"], c["meta"]
    B, nz = m["B"], m["nz"]
    Q.train()
    z = torch.from_numpy(synth.normal_f32(SEED_Z0, 0, (B, nz))).to(device)
    mask = torch.ones(B, 1, device=device)
    mask[1::3] = 0.0
    pe = synth.normal_f32(SEED_QT, 0, (B, nz))
    u = synth.uniform_f32(SEED_QT, 1, (B,), 0.0, 1.0)
    eps = synth.normal_f32(SEED_QT, 2, (B, nz))
    orig = torch.randn, torch.rand, torch.randn_like
    torch.randn = lambda *a, **k: torch.from_numpy(pe.copy()).to(k.get("device") or "cpu")
    torch.rand = lambda *a, **k: torch.from_numpy(u.copy())
    torch.randn_like = lambda t, **k: torch.from_numpy(eps.copy()).to(t.device)
    try:
        Q.zero_grad()
        loss = Q.calculate_loss(x=x, z=z, mask=mask)
        loss.mean().backward()
    finally:
        torch.randn, torch.rand, torch.randn_like = orig
    grads = [p.grad.detach().cpu().numpy() for p in Q.parameters() if p.grad is not None]
    return loss.detach().cpu().numpy(), grads, rec, meta


def build_q_case(name, device="cpu"):
    import torch

    from damc import synth
    from src import diffusion_net as dn

    rec, meta = load_golden(name)
    Q = dn._netQ_U(nc=meta["nc"], nz=meta["nz"], nxemb=meta["nxemb"], ntemb=meta["ntemb"], nif=meta["nif"],
                   diffusion_residual=True, n_interval=meta["n_interval"], logsnr_min=meta["logsnr_min"],
                   logsnr_max=meta["logsnr_max"], var_type=meta["var_type"], with_noise=True, cond_w=0.0,
                   net_arch="A", dataset=meta["dataset"])
    synth.load_into(Q, SEED_Q)
    Q.to(device).eval()
    B, nz, nc, H, n = meta["B"], meta["nz"], meta["nc"], meta["H"], meta["n_interval"]
    x = torch.from_numpy(synth.uniform_f32(SEED_X, 0, (B, nc, H, H))).to(device)
    zt0 = torch.from_numpy(synth.normal_f32(SEED_QN, 0, (B, nz))).to(device)
    pe_noise = torch.from_numpy(synth.normal_f32(SEED_QN, 1, (B, nz))).to(device)
    eps = torch.from_numpy(np.stack([synth.normal_f32(SEED_QN, 100 + i, (B, nz)) for i in range(max(n - 1, 1))]))
    return dict(Q=Q, x=x, zt0=zt0, pe_noise=pe_noise, eps=eps.to(device), rec=rec, meta=meta)


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch.device("cuda:0")
