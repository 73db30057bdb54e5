"""Run the HIP denoiser forward+backward of the Q update (bench config) N times, for rocprofv3 --stats."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "diffusion-amortized-mcmc_amd"))
import torch  # noqa: E402

from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

B = 128
p = synth.load_into(dn.Diffusion_UnetA(nz=128, nxemb=1024, ntemb=128, residual=True, nf=4), 3).cuda()
zt = torch.from_numpy(synth.normal_f32(5, 0, (B, 128))).cuda()
logsnr = torch.from_numpy(synth.uniform_f32(5, 1, (B,), -5.0, 9.0)).cuda()
xe = torch.from_numpy(synth.normal_f32(5, 2, (B, 1024))).cuda().requires_grad_(True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for _ in range(n):
    p(zt, logsnr.clone(), xe).square().sum().backward()
torch.cuda.synchronize()
ts = []
for _ in range(n):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    p(zt, logsnr.clone(), xe).square().sum().backward()
    b.record()
    b.synchronize()
    ts.append(a.elapsed_time(b))
print("denoiser fwd+bwd ms (median)", sorted(ts)[len(ts) // 2])
