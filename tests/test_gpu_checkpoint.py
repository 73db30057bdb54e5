"""GPU: SURVEY.md §8(f) row 4 on the HIP path — a checkpoint in the reference's training format
(train_gen_recon.py:284-294, loaded as in train_gen_recon.py:163-170 / eval_gen_recon.py:156-163), written by
the reference's own modules and optimisers (tests/golden/make_golden.py), loads into the drop-in modules on the
GPU and the HIP kernels reproduce the reference's outputs of the loaded nets (gen_x, ebm_e, xemb in
ckpt_cifar10_tiny.npz) and the oracle's posterior step and reverse sweep on them.

The checkpoint is loaded with weights_only=True.  Its nets are tiny (ngf=4: 32/16/8 channels, nif=2, nf=1):
layers whose channel counts the limb engine cannot gather run on the fp32 MFMA engine, so this also covers the
engine dispatch at widths the benchmark never uses.  Tolerances as tests/test_gpu_langevin.py."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ckpt(gpu_device):
    from src import diffusion_net as dn

    sd = torch.load(os.path.join(GOLDEN, "ckpt_cifar10_tiny.pth.tar"), weights_only=True, map_location="cpu")
    d = np.load(os.path.join(GOLDEN, "ckpt_cifar10_tiny.npz"))
    meta = json.loads(str(d["meta"]))
    nz = meta["nz"]
    G = dn._netG_cifar10(nz=nz, ngf=meta["ngf"], nc=3)
    E = dn._netE(nz=nz, ndf=meta["ndf"])
    Q = dn._netQ_U(**meta["q"])
    G.load_state_dict(sd["G_state_dict"])
    E.load_state_dict(sd["E_state_dict"])
    Q.load_state_dict(sd["Q_state_dict"])
    for m in (G, E, Q):
        m.to(gpu_device).eval()
    return dict(G=G, E=E, Q=Q, rec=d, meta=meta, nz=nz)


def _inputs(nz, device):
    from damc import synth

    x = torch.from_numpy(synth.uniform_f32(60, 0, (4, 3, 32, 32))).to(device)
    z = torch.from_numpy(synth.normal_f32(61, 0, (4, nz))).to(device)
    return x, z


def test_loaded_nets_reproduce_reference_outputs(ckpt, gpu_device):
    from damc import amortizer, langevin

    x, z = _inputs(ckpt["nz"], gpu_device)
    rec = ckpt["rec"]
    assert rel_l2(langevin.generator_forward(z, ckpt["G"]).cpu().numpy(), rec["gen_x"]) < 1e-5
    e, _ = langevin.ebm_energy_grad(z, ckpt["E"])
    assert rel_l2(e.cpu().numpy(), rec["ebm_e"]) < 1e-5
    assert rel_l2(amortizer.encoder_forward(ckpt["Q"].encoder, x).cpu().numpy(), rec["xemb"]) < 1e-5


def test_loaded_nets_langevin_and_sweep_vs_oracle(ckpt, gpu_device):
    from damc import amortizer, langevin
    from oracle import damc_oracle as orc

    x, z0 = _inputs(ckpt["nz"], gpu_device)
    G, E, Q = ckpt["G"], ckpt["E"], ckpt["Q"]
    L, P = orc.generator_layers(G.cpu()), orc.ebm_params(E.cpu())
    G.to(gpu_device), E.to(gpu_device)
    noise = torch.from_numpy(np.random.default_rng(5).standard_normal((10, 4, ckpt["nz"])).astype(np.float32))
    z = z0.clone()
    langevin.posterior_langevin(z, x, G, E, 1, 0.1, 0.1, False)
    want = orc.posterior_langevin(L, P, z0.cpu(), x.cpu(), 1, 0.1, 0.1).numpy()
    assert rel_l2(z.cpu().numpy(), want) < 1e-6
    z = z0.clone()
    langevin.posterior_langevin(z, x, G, E, 10, 0.1, 0.1, True, noise=noise.to(gpu_device))
    want = orc.posterior_langevin(L, P, z0.cpu(), x.cpu(), 10, 0.1, 0.1, noise=noise).numpy()
    assert rel_l2(z.cpu().numpy(), want) < 2e-4
    # Q(x): encoder + the whole n_interval-step reverse sweep with injected noise
    m = ckpt["meta"]["q"]
    xemb = amortizer.encoder_forward(Q.encoder, x)
    zt0 = torch.from_numpy(np.random.default_rng(6).standard_normal((4, ckpt["nz"])).astype(np.float32))
    eps = torch.from_numpy(np.random.default_rng(7).standard_normal((m["n_interval"] - 1, 4, ckpt["nz"]))
                           .astype(np.float32))
    zt = zt0.to(gpu_device)
    amortizer.reverse_sweep(Q, xemb, zt, noise=eps.to(gpu_device))
    Qc = ckpt["Q"].cpu()
    want, _ = orc.reverse_sweep(Qc, orc.encoder_forward(Qc.encoder, x.cpu()), zt0, eps, m["n_interval"],
                                m["logsnr_min"], m["logsnr_max"], m["var_type"])
    Q.to(gpu_device)
    assert rel_l2(zt.cpu().numpy(), want.numpy()) < 1e-4
