"""GPU: one trimmed training iteration of workspace/train_gen_recon.py:179-261 and the eval MSE loop
(:324-348) run through the drop-in ``src`` package with tiny widths — the drivers' call pattern,
unchanged, on the HIP path."""
import pytest
import torch
import torch.optim as optim

pytestmark = pytest.mark.gpu


def test_train_iteration_and_eval_mse(gpu_device):
    from src import diffusion_net as dn
    from src.MCMC import gen_samples_with_diffusion_prior, sample_langevin_post_z_with_prior, sample_langevin_prior_z

    torch.manual_seed(1)
    nz = 128
    G = dn._netG_cifar10(nz=nz, ngf=16, nc=3).cuda()
    Q = dn._netQ_U(nc=3, nz=nz, nxemb=64, ntemb=32, nif=8, diffusion_residual=True, n_interval=10,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset="cifar10").cuda()
    Q_dummy = dn._netQ_U(nc=3, nz=nz, nxemb=64, ntemb=32, nif=8, diffusion_residual=True, n_interval=10,
                         logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0,
                         net_arch="A", dataset="cifar10").cuda()
    for p, tp in zip(Q.parameters(), Q_dummy.parameters()):
        tp.data.copy_(p.data)
    E = dn._netE(nz=nz).cuda()
    G_opt = optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
    Q_opt = optim.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
    E_opt = optim.Adam(E.parameters(), lr=1e-4, betas=(0.5, 0.999))
    x = torch.rand(8, 3, 32, 32, device=gpu_device) * 2 - 1

    for _ in range(2):
        z_mask = (torch.rand(len(x), device=x.device) >= 0.2).float().unsqueeze(-1)
        Q.eval(), G.eval(), E.eval()
        with torch.no_grad():
            z0 = Q_dummy(x)
            zp = Q(x=None, b=x.size(0), device=x.device)
        assert zp.shape == (8, nz)
        zk_pos, zk_neg = z0.detach().clone(), z0.detach().clone()
        zk_pos.requires_grad = True
        zk_neg.requires_grad = True
        zk_pos = sample_langevin_post_z_with_prior(z=zk_pos, x=x, netG=G, netE=E, g_l_steps=5, g_llhd_sigma=0.1,
                                                   g_l_with_noise=True, g_l_step_size=0.1, verbose=False)
        zk_neg = sample_langevin_prior_z(z=torch.cat([zk_neg, torch.randn_like(zk_neg, requires_grad=True)], dim=0),
                                         netE=E, e_l_steps=10, e_l_step_size=0.4, e_l_with_noise=True, verbose=False)
        for __ in range(2):
            Q_opt.zero_grad()
            Q.train()
            Q.calculate_loss(x=x, z=zk_pos, mask=z_mask).mean().backward()
            Q_opt.step()
        G_opt.zero_grad()
        G.train()
        g_loss = torch.sum((G(zk_pos) - x) ** 2, dim=[1, 2, 3]).mean()
        g_loss.backward()
        G_opt.step()
        E_opt.zero_grad()
        E.train()
        (E(zk_pos).mean() - E(zk_neg).mean()).backward()
        E_opt.step()
        for p, tp in zip(Q.parameters(), Q_dummy.parameters()):
            tp.data.copy_(0.005 * p.data + 0.995 * tp.data)
        assert torch.isfinite(zk_pos).all() and torch.isfinite(zk_neg).all() and torch.isfinite(g_loss)

    # eval MSE (train_gen_recon.py:324-348): Q(x) -> 10 no-noise posterior steps -> mean SE
    Q.eval(), G.eval(), E.eval()
    with torch.no_grad():
        z0 = Q(x)
    zk = z0.detach().clone().requires_grad_(True)
    zk = sample_langevin_post_z_with_prior(z=zk, x=x, netG=G, netE=E, g_l_steps=10, g_llhd_sigma=0.1,
                                           g_l_with_noise=False, g_l_step_size=0.1, verbose=False)
    with torch.no_grad():
        mse_hip = torch.mean((G(zk) - x) ** 2, dim=[1, 2, 3]).sum().item()
    assert mse_hip == mse_hip and mse_hip > 0
    xs, zs = gen_samples_with_diffusion_prior(b=4, device=x.device, netQ=Q, netG=G)
    assert xs.shape == (4, 3, 32, 32)


def test_sharded_recon_mse_single_rank(gpu_device):
    """damc.dist.sharded_recon_mse on one rank == the driver's eval loop."""
    from damc import dist as ddist
    from damc import synth
    from src import diffusion_net as dn

    torch.manual_seed(3)
    G = synth.load_into(dn._netG_cifar10(nz=128, ngf=16, nc=3), 0).cuda().eval()
    E = synth.load_into(dn._netE(nz=128), 10).cuda().eval()
    Q = dn._netQ_U(nc=3, nz=128, nxemb=64, ntemb=32, nif=8, diffusion_residual=True, n_interval=5,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=False, dataset="cifar10")
    synth.load_into(Q, 20)
    Q.cuda().eval()
    batches = [torch.rand(6, 3, 32, 32, device=gpu_device) * 2 - 1 for _ in range(2)]
    mse = ddist.sharded_recon_mse(Q, G, E, batches, g_l_steps=3)
    # same computation through the drop-in API (Q sweep is deterministic with with_noise=False
    # except for its initial zt draw, so re-seed identically)
    torch.manual_seed(3)
    from src.MCMC import sample_langevin_post_z_with_prior

    tot, n = 0.0, 0
    for x in batches:
        with torch.no_grad():
            z = Q(x)
        z = sample_langevin_post_z_with_prior(z.requires_grad_(True), x, G, E, 3, 0.1, False, 0.1)
        with torch.no_grad():
            tot += torch.mean((G(z) - x) ** 2, dim=[1, 2, 3]).sum().item()
        n += len(x)
    assert abs(mse - tot / n) < 1e-5 * max(1.0, tot / n)
