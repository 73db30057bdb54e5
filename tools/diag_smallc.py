# accuracy of the k4 s2 output layer path (SMALLC) vs k3 s1, in tiny 2-3 layer generators, against fp64
import os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "tests"), os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch
from conftest import rel_l2
from damc import synth, langevin as lv
from oracle import damc_oracle as orc
dev = torch.device("cuda:0")

class Gen(torch.nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.gen = torch.nn.Sequential(*layers)

def make(nz, C, last_k, up=0, hw0=4):
    L = [torch.nn.ConvTranspose2d(nz, C, hw0, 1, 0), torch.nn.LeakyReLU(0.2)]
    for _ in range(up):
        L += [torch.nn.ConvTranspose2d(C, C, 4, 2, 1), torch.nn.LeakyReLU(0.2)]
    L += [torch.nn.ConvTranspose2d(C, 3, 4, 2, 1) if last_k == 4 else torch.nn.ConvTranspose2d(C, 3, 3, 1, 1),
          torch.nn.Tanh()]
    return synth.load_into(Gen(L), 0).to(dev).eval()

for nz, C, k, up, B in ((128, 128, 4, 0, 16), (128, 128, 3, 0, 16), (128, 128, 4, 1, 16), (128, 128, 3, 1, 16),
                        (128, 64, 4, 2, 32), (100, 128, 4, 1, 32), (128, 256, 4, 2, 8)):
    G = make(nz, C, k, up)
    hw = G.gen[-2].stride[0] * (4 * 2 ** up) if k == 4 else 4 * 2 ** up
    x = torch.rand(B, 3, hw, hw, device=dev) * 2 - 1
    z = torch.randn(B, nz, device=dev)
    L32, L64 = orc.generator_layers(G), orc.generator_layers(G, torch.float64)
    g = lv.likelihood_grad(z, x, G, 0.1).cpu().numpy()
    g64 = orc.likelihood_grad(L64, z.cpu().double(), x.cpu().double(), 0.1)[0].numpy()
    g32 = orc.likelihood_grad(L32, z.cpu(), x.cpu(), 0.1)[0].numpy()
    xh = lv.generator_forward(z, G).cpu().numpy()
    x64 = orc.generator_sample(L64, z.cpu().double()).numpy()
    print("nz %d C %d last k%d, %d up layers, B=%d: lik grad %.2e (fp32 ref %.2e)  G(z) %.2e" % (
        nz, C, k, up, B, rel_l2(g, g64), rel_l2(g32, g64), rel_l2(xh, x64)))
