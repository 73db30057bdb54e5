"""Q update legs (workspace/train_gen_recon.py:211-220) at the bench config, stock PyTorch: encoder fwd+bwd,
denoiser loss fwd+bwd, optimiser, timed with HIP events (median of 5)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "diffusion-amortized-mcmc_amd"))
import torch  # noqa: E402
import torch.optim as optim  # noqa: E402

from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

B, nz = 128, 128
dev = torch.device("cuda")
qa = dict(nc=3, nz=nz, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100, logsnr_min=-5.1,
          logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A", dataset="cifar10")
Q = synth.load_into(dn._netQ_U(**qa), 20).to(dev).train()
opt = optim.AdamW(Q.parameters(), weight_decay=1e-4, lr=2e-4, betas=(0.5, 0.999))
x = torch.from_numpy(synth.uniform_f32(1, 0, (B, 3, 32, 32))).to(dev)
z = torch.from_numpy(synth.normal_f32(2, 0, (B, nz))).to(dev)
mask = torch.ones(B, 1, device=dev)
xe = torch.randn(B, 1024, device=dev, requires_grad=True)


def med(fn, n=7):
    fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return round(sorted(ts)[len(ts) // 2], 3)


def enc():
    Q.encoder(x).sum().backward()


def den():
    u = torch.rand(B, device=dev)
    from src.diffusion_helper_func import logsnr_schedule_fn
    ls = logsnr_schedule_fn(u, logsnr_max=9.8, logsnr_min=-5.1)
    Q.p(z=z, logsnr=ls, xemb=xe).square().sum().backward()


def full():
    opt.zero_grad()
    Q.calculate_loss(x=x, z=z, mask=mask).mean().backward()
    torch.nn.utils.clip_grad_norm_(Q.parameters(), max_norm=100)
    opt.step()


def step_only():
    torch.nn.utils.clip_grad_norm_(Q.parameters(), max_norm=100)
    opt.step()


print({"encoder_fwd_bwd_ms": med(enc), "denoiser_fwd_bwd_ms": med(den), "q_update_ms": med(full),
       "clip_and_adamw_ms": med(step_only)})
