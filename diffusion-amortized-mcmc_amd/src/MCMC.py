"""Drop-in for workspace/src/MCMC.py: the reference's sampling API on the MI355X HIP path.

``train_gen_recon.py`` / ``eval_gen_recon.py`` import these names unchanged.  Semantics kept
from the reference:
  * z is updated in place (the caller's leaf tensor sees the new values) and ``z.detach()``
    is returned (MCMC.py:46,74);
  * the nets' ``requires_grad`` is switched off during the call and back ON afterwards
    (MCMC.py:30,45,51-52,72-73), even if it was off before;
  * the verbose log string has the reference's format; the per-step host syncs of the
    reference (``.item()`` every step) happen only when ``verbose`` is set;
  * noise comes from in-kernel Philox keyed by a seed drawn from torch's generator, so
    ``torch.manual_seed`` still makes a run reproducible (bitwise parity with torch's CUDA
    RNG stream is neither possible nor required).
"""
import torch

from damc import langevin as _lv


def set_requires_grad(nets, requires_grad=False):
    """Toggle ``requires_grad`` of every parameter of a net or a list of nets (MCMC.py:12-25)."""
    for net in nets if isinstance(nets, list) else [nets]:
        if net is not None:
            for p in net.parameters():
                p.requires_grad = requires_grad


def _as_work_tensor(z):
    """In-place target: z itself when it is contiguous fp32 on the GPU, else a working copy."""
    zd = z.detach()
    if zd.dtype == torch.float32 and zd.is_contiguous() and zd.device.type == "cuda":
        return zd, False
    return zd.to(dtype=torch.float32).contiguous().clone(), True


def sample_langevin_prior_z(z, netE, e_l_steps, e_l_step_size, e_l_with_noise, verbose=False):
    """Prior Langevin on U(z) = sum E(z) + |z|^2/2 — all steps in one HIP launch."""
    set_requires_grad(netE, requires_grad=False)
    work, copied = _as_work_tensor(z)
    diag = _lv.prior_langevin(work, netE, e_l_steps, e_l_step_size, e_l_with_noise, diag=verbose)
    if copied:
        z.data = work.to(z.dtype)
    if verbose:
        d = diag.cpu().tolist()
        msg = "Step/en/z_norm: "
        for i in range(e_l_steps):
            if i % 5 == 0 or i == e_l_steps - 1:
                msg += "{}/{:.3f}/{:.3f}  ".format(i, d[i][0], d[i][1])
        print("Log prior sampling.")
        print(msg)
    set_requires_grad(netE, requires_grad=True)
    return z.detach()


def sample_langevin_post_z_with_prior(z, x, netG, netE, g_l_steps, g_llhd_sigma, g_l_with_noise, g_l_step_size,
                                      verbose=False):
    """Posterior Langevin on U(z) = |G(z)-x|^2/(2 sigma^2) + sum E(z) + |z|^2/2 on the HIP path."""
    set_requires_grad(netG, requires_grad=False)
    set_requires_grad(netE, requires_grad=False)
    work, copied = _as_work_tensor(z)
    diag = _lv.posterior_langevin(work, x, netG, netE, g_l_steps, g_llhd_sigma, g_l_step_size, g_l_with_noise,
                                  diag=verbose)
    if copied:
        z.data = work.to(z.dtype)
    if verbose:
        d = diag.cpu().tolist()
        msg = "Step/cross_entropy/recons_loss: "
        for i in range(g_l_steps):
            msg += "{}/{:.3f}/{:.3f}/{:.3f}/{:.8f}  ".format(i, d[i][0], d[i][1], d[i][2], d[i][3])
        print("Log posterior sampling.")
        print(msg)
    set_requires_grad(netG, requires_grad=True)
    set_requires_grad(netE, requires_grad=True)
    return z.detach()


def sample_invert_z(z, x, netG, netF, netE, g_l_steps, g_l_step_size, verbose=False):
    """StyleGAN inversion (Adam, not Langevin) is outside the hot path."""
    raise NotImplementedError("sample_invert_z (StyleGAN inversion) is not part of the MI355X hot path")


def gen_samples(bs, nz, netE, netG, e_l_steps, e_l_step_size, e_l_with_noise):
    """z ~ N(0, I) -> prior Langevin -> G(z) under no_grad (MCMC.py:119-128)."""
    zk = torch.randn(bs, nz).cuda()
    zk.requires_grad = True
    zk = sample_langevin_prior_z(z=zk, netE=netE, e_l_steps=e_l_steps, e_l_step_size=e_l_step_size,
                                 e_l_with_noise=e_l_with_noise, verbose=False)
    with torch.no_grad():
        return _lv.generator_forward(zk, netG)


def gen_samples_with_diffusion_prior(b, device, netQ, netG):
    """Q(x=None, b) reverse sweep -> G(z) under no_grad (MCMC.py:146-150)."""
    with torch.no_grad():
        zk = netQ(x=None, b=b, device=device)
        return _lv.generator_forward(zk, netG), zk


def _fid(fid_samples, real_m, real_s, save_name):
    """pfw.fid(samples, real_m, real_s) (MCMC.py:136-139) with the statistics on the HIP path: Inception pool
    features (pytorch-fid, third-party: SURVEY.md §8c, FID parity unpinned) -> damc_fid_accumulate (fp64
    sum f / sum f f^T on the device) -> mu, sigma -> pytorch-fid's Frechet distance (damc.fid)."""
    from damc import fid as _dfid

    fid_samples = torch.cat(fid_samples, dim=0)
    fid_samples = (1.0 + torch.clamp(fid_samples, min=-1.0, max=1.0)) / 2.0
    # the samples' own device when they are on a GPU (the reference's pfw.fid used cuda:0, MCMC.py:139); no
    # collective: a driver that computes FID on one rank must not block on the others
    dev = fid_samples.device if fid_samples.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
    fid = _dfid.fid_of_samples(fid_samples.to(dev), real_m, real_s)
    if save_name is not None:
        import torchvision

        torchvision.utils.save_image(fid_samples[:64].clone().detach().cpu(), save_name, normalize=True, nrow=8)
    return fid


def calculate_fid(n_samples, nz, netE, netG, e_l_steps, e_l_step_size, e_l_with_noise, real_m, real_s, save_name,
                  bs=500):
    samples = [gen_samples(bs, nz, netE, netG, e_l_steps, e_l_step_size, e_l_with_noise).detach().clone()
               for _ in range(n_samples // bs)]
    return _fid(samples, real_m, real_s, save_name)


def calculate_fid_with_diffusion_prior(n_samples, device, netQ, netG, netE, real_m, real_s, save_name, bs=500):
    samples = [gen_samples_with_diffusion_prior(bs, device, netQ, netG)[0].detach().clone()
               for _ in range(n_samples // bs)]
    return _fid(samples, real_m, real_s, save_name)


def calculate_fid_with_samples(fid_samples, real_m, real_s, save_name):
    return _fid(fid_samples, real_m, real_s, save_name)
