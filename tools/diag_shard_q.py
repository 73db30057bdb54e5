"""Where does a sharded Q(x) leave the whole-batch one?  Encoder xemb and the reverse sweep compared separately,
B vs 8 x B/8 (run through gpurun): prints the max |diff| and the number of differing rows per stage."""
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "diffusion-amortized-mcmc_amd"))

import torch  # noqa: E402

from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402


def cmp(name, a, b):
    d = (a - b).abs()
    rows = int((a != b).reshape(len(a), -1).any(dim=1).sum())
    print("%-40s max|diff| %.3e  rows differing %d / %d" % (name, float(d.max()), rows, len(a)), flush=True)


def main(dataset, hw, bsz, nint=100):
    dev = torch.device("cuda")
    Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=nint,
                   logsnr_min=-5.1, logsnr_max=9.8, var_type="large", with_noise=True, cond_w=0.0, net_arch="A",
                   dataset=dataset)
    synth.load_into(Q, 20)
    Q.to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(81, 0, (bsz, 3, hw, hw))).to(dev)
    zt0 = torch.from_numpy(synth.normal_f32(82, 0, (bsz, 128))).to(dev)
    s = bsz // 8
    with torch.no_grad():
        xa = amortizer.encoder_forward(Q.encoder, x)
        xs = torch.cat([amortizer.encoder_forward(Q.encoder, x[s * r:s * r + s].contiguous()) for r in range(8)])
        cmp("%s encoder xemb B=%d vs 8x%d" % (dataset, bsz, s), xs, xa)
        for env in ({}, {"DAMC_SWEEP_TEAM": "0"}, {"DAMC_SWEEP_HYPER": "fp32"},
                    {"DAMC_SWEEP_TEAM": "0", "DAMC_SWEEP_HYPER": "fp32"}):
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            za = zt0.clone()
            amortizer.reverse_sweep(Q, xa, za, seed=9)
            parts = []
            for r in range(8):
                zb = zt0[s * r:s * r + s].clone()
                amortizer.reverse_sweep(Q, xa[s * r:s * r + s].contiguous(), zb, seed=9, chain_base=s * r)
                parts.append(zb)
            cmp("%s sweep %s B=%d vs 8x%d" % (dataset, env or "default", bsz, s), torch.cat(parts), za)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main("cifar10", 32, 128, 10)
    main("celebaHQ", 256, 64, 10)
