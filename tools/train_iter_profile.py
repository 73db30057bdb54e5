"""Time the legs of one reference training iteration (workspace/train_gen_recon.py:179-241) at the bench
config (CIFAR-10, B=128, nz=128, ngf=128, Q: nif 64, nxemb 1024, ntemb 128, 100 steps) on the drop-in
package: Q(x) amortizer forwards, the Langevin block, 6 Q updates, the G update, the E update.
--damc-optim: the three optimisers and their clip_grad_norm_ on damc.optim (fused clip + Adam/AdamW)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "diffusion-amortized-mcmc_amd"))
import torch  # noqa: E402
import torch.optim as optim  # noqa: E402

from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402
from src.MCMC import sample_langevin_post_z_with_prior, sample_langevin_prior_z  # noqa: E402

B, nz = 128, 128
dev = torch.device("cuda")
G = synth.load_into(dn._netG_cifar10(nz=nz, ngf=128, nc=3), 0).to(dev)
E = synth.load_into(dn._netE(nz=nz), 10).to(dev)
qa = dict(nc=3, nz=nz, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100, logsnr_min=-5.1,
          logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A", dataset="cifar10")
Q = synth.load_into(dn._netQ_U(**qa), 20).to(dev)
Qd = synth.load_into(dn._netQ_U(**qa), 20).to(dev)
DAMC_OPTIM = "--damc-optim" in sys.argv
if DAMC_OPTIM:
    from damc import optim  # noqa: E402,F811
G_opt = optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.999))
Q_opt = optim.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
E_opt = optim.Adam(E.parameters(), lr=1e-4, betas=(0.5, 0.999))


def clip_step(opt, params, max_norm=100):
    if DAMC_OPTIM:
        opt.clip_and_step(max_norm)
    else:
        torch.nn.utils.clip_grad_norm_(params, max_norm=max_norm)
        opt.step()
x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, 32, 32))).to(dev)


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def iteration(t):
    z_mask = (torch.rand(B, device=dev) >= 0.2).float().unsqueeze(-1)
    Q.eval(), G.eval(), E.eval()
    e0 = ev()
    with torch.no_grad():
        z0 = Qd(x)
        zp = Q(x=None, b=B, device=dev)
    e1 = ev()
    zk_pos, zk_neg = z0.detach().clone(), z0.detach().clone()
    zk_pos.requires_grad = True
    zk_neg.requires_grad = True
    zk_pos = sample_langevin_post_z_with_prior(z=zk_pos, x=x, netG=G, netE=E, g_l_steps=30, g_llhd_sigma=0.1,
                                               g_l_with_noise=True, g_l_step_size=0.1)
    zk_neg = sample_langevin_prior_z(z=torch.cat([zk_neg, torch.randn_like(zk_neg, requires_grad=True)], dim=0),
                                     netE=E, e_l_steps=60, e_l_step_size=0.4, e_l_with_noise=True)
    e2 = ev()
    for __ in range(6):
        Q_opt.zero_grad()
        Q.train()
        Q.calculate_loss(x=x, z=zk_pos, mask=z_mask).mean().backward()
        clip_step(Q_opt, Q.parameters())
    e3 = ev()
    G_opt.zero_grad()
    G.train()
    g_loss = torch.sum((G(zk_pos) - x) ** 2, dim=[1, 2, 3]).mean()
    g_loss.backward()
    clip_step(G_opt, G.parameters())
    e4 = ev()
    E_opt.zero_grad()
    E.train()
    (E(zk_pos).mean() - E(zk_neg).mean()).backward()
    clip_step(E_opt, E.parameters())
    e5 = ev()
    torch.cuda.synchronize()
    evs = [e0, e1, e2, e3, e4, e5]
    names = ["q_forwards", "langevin", "q_updates_x6", "g_update", "e_update"]
    for n, a, b in zip(names, evs[:-1], evs[1:]):
        t.setdefault(n, []).append(a.elapsed_time(b))
    t.setdefault("total", []).append(e0.elapsed_time(e5))


t = {}
for i in range(4):
    iteration(t if i > 0 else {})
print({k: round(sorted(v)[len(v) // 2], 2) for k, v in t.items()})
