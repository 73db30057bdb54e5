"""Run the HIP G update (bench.g_update_bench's step) a few times, for rocprofv3 --kernel-trace --stats."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "diffusion-amortized-mcmc_amd"))
import torch  # noqa: E402

from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

B, NZ = 128, 128
G = synth.load_into(dn._netG_cifar10(nz=NZ, ngf=128, nc=3), 0).cuda().train()
z = torch.from_numpy(synth.normal_f32(41, 0, (B, NZ))).cuda()
x = torch.from_numpy(synth.uniform_f32(42, 0, (B, 3, 32, 32))).cuda()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    G.zero_grad(set_to_none=True)
    torch.sum((G(z) - x) ** 2, dim=[1, 2, 3]).mean().backward()
torch.cuda.synchronize()
print("ok")
