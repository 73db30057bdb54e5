"""CPU: the oracle (oracle/damc_oracle.py) against the reference's golden vectors.

Tolerances (~4x the reference's own fp32-vs-fp64 / thread-count spread):
  1 posterior step rel-L2(z) <= 1e-6;  10 steps (no noise) <= 2e-4;  30 steps <= 2e-3;
  recon MSE rel <= 1e-5;  60 prior steps <= 1e-4;  gradients rel-L2 <= 1e-5.
"""
import numpy as np
import pytest
import torch

from conftest import (G_NAMES, Q_END_TOL, Q_NAMES, build_g_case, build_q_case, gtrain_check, gtrain_inputs,
                      load_golden, qtrain_run, rel_l2)
from oracle import damc_oracle as orc

torch.set_num_threads(8)

FAST_G = [n for n in G_NAMES if n != "celebaHQ_w8"]


@pytest.mark.parametrize("name", G_NAMES)
def test_state_dict_keys_match_reference(name):
    c = build_g_case(name)
    assert [[k, list(v.shape)] for k, v in c["G"].state_dict().items()] == c["meta"]["g_keys"]
    assert [[k, list(v.shape)] for k, v in c["E"].state_dict().items()] == c["meta"]["e_keys"]


@pytest.mark.parametrize("name", Q_NAMES)
def test_q_state_dict_keys_match_reference(name):
    c = build_q_case(name)
    assert [[k, list(v.shape)] for k, v in c["Q"].state_dict().items()] == c["meta"]["q_keys"]


@pytest.mark.parametrize("name", G_NAMES)
def test_generator_forward_and_grads(name):
    c = build_g_case(name)
    L = orc.generator_layers(c["G"])
    xh = orc.generator_sample(L, c["z0"]).numpy()
    if "gen_x" in c["rec"]:
        assert rel_l2(xh, c["rec"]["gen_x"]) < 1e-6
    else:
        assert rel_l2(xh[:, :, ::4, ::4], c["rec"]["gen_x_sub4"]) < 1e-6
    sigma = c["meta"]["sigma"]
    gl, lik, _ = orc.likelihood_grad(L, c["z0"], c["x"], sigma)
    assert rel_l2(gl.numpy(), c["rec"]["lik_grad0"]) < 1e-5
    assert abs(float(lik) - float(c["rec"]["lik0"])) / float(c["rec"]["lik0"]) < 1e-5
    e, ge = orc.ebm_energy_grad(orc.ebm_params(c["E"]), c["z0"])
    assert rel_l2(e.numpy(), c["rec"]["ebm_e"]) < 1e-6
    assert rel_l2(ge.numpy(), c["rec"]["ebm_grad0"]) < 1e-5


@pytest.mark.parametrize("name", G_NAMES)
def test_generator_train_grads(name):
    """G update (train_gen_recon.py:222-231): the oracle's explicit backward vs the reference's autograd."""
    G, z0, x, rec, meta = gtrain_inputs(name)
    L = orc.generator_layers(G)
    xh = orc.generator_sample(L, z0)
    gx = 2.0 * (xh - x) / meta["B"]
    loss = float(((xh - x) ** 2).sum(dim=(1, 2, 3)).mean())
    assert abs(loss - float(rec["g_loss"])) / float(rec["g_loss"]) < 1e-6
    grads, _, _ = orc.generator_train_grads(L, z0, gx)
    flat = [t for gw, gb in grads for t in ((gw,) if gb is None else (gw, gb))]
    gtrain_check([t.numpy() for t in flat], rec, meta, 1e-5)


@pytest.mark.parametrize("name", FAST_G)
def test_posterior_langevin(name):
    c = build_g_case(name)
    L, P = orc.generator_layers(c["G"]), orc.ebm_params(c["E"])
    m = c["meta"]
    z1 = orc.posterior_langevin(L, P, c["z0"], c["x"], 1, m["sigma"], m["step"])
    assert rel_l2(z1.numpy(), c["rec"]["post_z1"]) < 1e-6
    z10 = orc.posterior_langevin(L, P, c["z0"], c["x"], 10, m["sigma"], m["step"])
    assert rel_l2(z10.numpy(), c["rec"]["post_z10"]) < 2e-4
    mse = ((orc.generator_sample(L, z10) - c["x"]) ** 2).mean(dim=(1, 2, 3)).numpy()
    assert np.max(np.abs(mse - c["rec"]["recon_mse10"]) / c["rec"]["recon_mse10"]) < 1e-5
    z30 = orc.posterior_langevin(L, P, c["z0"], c["x"], 30, m["sigma"], m["step"], noise=c["post_noise"])
    assert rel_l2(z30.numpy(), c["rec"]["post_z30"]) < 2e-3


@pytest.mark.parametrize("name", ["cifar10_w16", "svhn_w16", "mnist_w16"])
def test_prior_langevin(name):
    c = build_g_case(name)
    P = orc.ebm_params(c["E"])
    z5 = orc.prior_langevin(P, c["zp0"], 5, c["meta"]["prior_step"])
    assert rel_l2(z5.numpy(), c["rec"]["prior_z5"]) < 1e-6
    z60 = orc.prior_langevin(P, c["zp0"], 60, c["meta"]["prior_step"], noise=c["prior_noise"])
    assert rel_l2(z60.numpy(), c["rec"]["prior_z60"]) < 1e-4


def test_toy_posterior():
    """Toy config #1: MLP G, E == 0, sigma = .25, 1000 steps (toy_example.py:110-131)."""
    from damc import synth
    from damc.toy import ToyG

    rec, meta = load_golden("toy")
    G = synth.load_into(ToyG(), 0)
    L = orc.generator_layers(G)
    B, nz = meta["B"], meta["nz"]
    z0 = torch.from_numpy(synth.normal_f32(2, 0, (B, nz)))
    x = torch.from_numpy(rec["x"])
    noise = torch.from_numpy(np.stack([synth.normal_f32(3, 100 + i, (B, nz)) for i in range(meta["steps"])]))
    z1 = orc.posterior_langevin(L, None, z0, x, 1, meta["sigma"], meta["step"], noise=noise, ebm_on=False)
    assert rel_l2(z1.numpy(), rec["post_z1"]) < 1e-6
    zN = orc.posterior_langevin(L, None, z0, x, meta["steps"], meta["sigma"], meta["step"], noise=noise,
                                ebm_on=False)
    assert rel_l2(zN.numpy(), rec["post_z1000"]) < 2e-3


@pytest.mark.parametrize("name", Q_NAMES)
def test_encoder_and_sweep(name):
    c = build_q_case(name)
    Q, m, rec = c["Q"], c["meta"], c["rec"]
    with torch.no_grad():
        xemb = orc.encoder_forward(Q.encoder, c["x"])
        assert rel_l2(xemb.numpy(), rec["xemb"]) < 1e-5
        zt, eps_log = orc.reverse_sweep(Q, xemb, c["zt0"], c["eps"], m["n_interval"], m["logsnr_min"],
                                        m["logsnr_max"], m["var_type"])
        # step 0 sees identical inputs (tight); later steps inherit the sweep's amplified
        # rounding (x sqrt(1+e^-l) up to ~13x per step)
        for k in range(3):
            assert rel_l2(eps_log[k].numpy(), rec["q_post_eps3"][k]) < (1e-5 if k == 0 else 1e-4)
        # short sweeps are ill-conditioned: the end-point is checked at 2x the reference's own
        # fp32 rounding spread (conftest.Q_END_TOL); the sharp check is eps at step 0 above
        tol_end = Q_END_TOL[name]
        assert rel_l2(zt.numpy(), rec["q_post"]) < tol_end
        pe = orc.prior_embedding(Q, c["pe_noise"])
        zt, eps_log = orc.reverse_sweep(Q, pe, c["zt0"], c["eps"], m["n_interval"], m["logsnr_min"],
                                        m["logsnr_max"], m["var_type"])
        assert rel_l2(eps_log[0].numpy(), rec["q_prior_eps3"][0]) < 1e-5
        assert rel_l2(zt.numpy(), rec["q_prior"]) < tol_end


def test_reference_checkpoint_loads():
    """a checkpoint written by the reference's training driver format
    (train_gen_recon.py:284-294: G/Q/Q_dummy/E state dicts + Adam/AdamW optimizer states + iter) loads
    unchanged into the drop-in modules and optimizers (train_gen_recon.py:163-170, eval_gen_recon.py:156-163),
    and the loaded nets reproduce the reference's outputs.  Loaded with weights_only=True."""
    import json
    import os

    import torch.optim as optim

    from conftest import GOLDEN
    from damc import synth
    from src import diffusion_net as dn

    sd = torch.load(os.path.join(GOLDEN, "ckpt_cifar10_tiny.pth.tar"), weights_only=True)
    d = np.load(os.path.join(GOLDEN, "ckpt_cifar10_tiny.npz"))
    meta = json.loads(str(d["meta"]))
    nz = meta["nz"]
    G = dn._netG_cifar10(nz=nz, ngf=meta["ngf"], nc=3)
    E = dn._netE(nz=nz, ndf=meta["ndf"])
    Q, Q_dummy = dn._netQ_U(**meta["q"]), dn._netQ_U(**meta["q"])
    G.load_state_dict(sd["G_state_dict"])
    Q.load_state_dict(sd["Q_state_dict"])
    Q_dummy.load_state_dict(sd["Q_dummy_state_dict"])
    E.load_state_dict(sd["E_state_dict"])
    G_opt = optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
    Q_opt = optim.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
    E_opt = optim.Adam(E.parameters(), lr=1e-4, betas=(0.5, 0.999))
    G_opt.load_state_dict(sd["G_optimizer"])
    Q_opt.load_state_dict(sd["Q_optimizer"])
    E_opt.load_state_dict(sd["E_optimizer"])
    assert sd["iter"] + 1 == 2
    assert len(G_opt.state) == len(list(G.parameters()))
    x = torch.from_numpy(synth.uniform_f32(60, 0, (4, 3, 32, 32)))
    z = torch.from_numpy(synth.normal_f32(61, 0, (4, nz)))
    with torch.no_grad():
        assert rel_l2(orc.generator_sample(orc.generator_layers(G), z).numpy(), d["gen_x"]) < 1e-6
        assert rel_l2(E(z).numpy(), d["ebm_e"]) < 1e-6
        assert rel_l2(orc.encoder_forward(Q.encoder, x).numpy(), d["xemb"]) < 1e-5


@pytest.mark.parametrize("name", ["q_cifar10_s", "q_svhn_s", "q_mnist_s", "q_cifar10_full", "q_celeba64_s", "q_celebaHQ_s"])
def test_q_update_loss_and_grads_cpu(name):
    """Q update (train_gen_recon.py:211-217) of the drop-in Q on CPU (stock ops) vs the reference's autograd."""
    loss, grads, rec, meta = qtrain_run(name, "cpu")
    assert rel_l2(loss, rec["loss"]) < 1e-6
    gtrain_check(grads, rec, meta, 1e-5)
