"""Split-K in-GEMM fix-up diagnostics (damc_x3_fixup_probe): per posterior step, the fix-up workgroups, waits that ran
out, bands the last arrivers took over and the wait times, at the per-rank batches (run through gpurun)."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib, langevin as lv, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

NETS = {"cifar10": ("_netG_cifar10", 128, 128, 32, 0.1), "svhn": ("_netG_svhn", 100, 64, 32, 0.1),
        "celeba64": ("_netG_celeba64", 100, 128, 64, 0.1), "celebaHQ": ("_netG_celebaHQ", 128, 128, 256, 1.0)}
os.environ["DAMC_X3_FIXUP"] = "1"  # the opt-in fix-up
dev = torch.device("cuda:0")
L = _lib.lib()
print("CUs:", torch.cuda.get_device_properties(0).multi_processor_count)
for case in sys.argv[1:] or ["cifar10:16", "svhn:64"]:
    net, B = case.split(":")[0], int(case.split(":")[1])
    ctor, nz, ngf, hw, sigma = NETS[net]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(dev).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(61, 0, (B, 3, hw, hw))).to(dev)
    z = torch.from_numpy(synth.normal_f32(62, 0, (B, nz))).to(dev)
    lv.posterior_langevin(z, x, G, E, 2, sigma, 0.1, True, seed=9)
    buf = torch.zeros(8, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    L.damc_x3_fixup_probe(buf.data_ptr())
    lv.posterior_langevin(z, x, G, E, 1, sigma, 0.1, True, seed=9)
    torch.cuda.synchronize()
    L.damc_x3_fixup_probe(None)
    s = [int(v) & 0xFFFFFFFF for v in buf.cpu().tolist()]
    nw = max(s[0] - s[5], 1)
    print("%s B=%d: fix-up workgroups %d, waits run out %d, bands taken over %d, last arrivers %d, wait max %.2f us "
          "mean %.2f us" % (net, B, s[0], s[1], s[2], s[5], s[3] / 100.0, s[4] / 100.0 / nw), flush=True)
