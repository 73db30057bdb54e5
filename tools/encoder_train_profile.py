"""HIP encoder forward+backward of the Q update (CIFAR-10 Encoder nif 64, nemb 1024, B=128) for rocprofv3."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "diffusion-amortized-mcmc_amd"))
import torch  # noqa: E402

from damc import synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

enc = synth.load_into(dn.Encoder_cifar10(nc=3, nemb=1024, nif=64), 4).cuda().train()
x = torch.from_numpy(synth.uniform_f32(6, 0, (128, 3, 32, 32))).cuda()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    enc.zero_grad(set_to_none=True)
    enc(x).square().sum().backward()
torch.cuda.synchronize()
print("ok")
