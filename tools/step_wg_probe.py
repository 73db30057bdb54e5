"""Per-workgroup start / K-loop end of every limb-engine launch of one posterior step (damc_clock_probe stamps,
100 MHz realtime; DAMC_CLOCK_REGIONS gives each launch its own slot region): where does a small-batch GEMM's time
go?  usage: python tools/step_wg_probe.py [net:B ...]   (default svhn:64 cifar10:16; run through gpurun)"""
import os
import sys

os.environ.setdefault("DAMC_CLOCK_REGIONS", "8")
import torch  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib, langevin as lv, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

NETS = {"cifar10": ("_netG_cifar10", 128, 128, 32, 0.1), "svhn": ("_netG_svhn", 100, 64, 32, 0.1),
        "celeba64": ("_netG_celeba64", 100, 128, 64, 0.1), "celebaHQ": ("_netG_celebaHQ", 128, 128, 256, 1.0)}
R, SLOTS = int(os.environ["DAMC_CLOCK_REGIONS"]), 4096
dev = torch.device("cuda:0")
L = _lib.lib()
q = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
for case in (sys.argv[1:] or ["svhn:64", "cifar10:16"]):
    net, B = case.split(":")[0], int(case.split(":")[1])
    ctor, nz, ngf, hw, sigma = NETS[net]
    G = synth.load_into(getattr(dn, ctor)(nz=nz, ngf=ngf, nc=3), 0).to(dev).eval()
    E = synth.load_into(dn._netE(nz=nz), 10).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(61, 0, (B, 3, hw, hw))).to(dev)
    z = torch.from_numpy(synth.normal_f32(62, 0, (B, nz))).to(dev)
    lv.posterior_langevin(z, x, G, E, 3, sigma, 0.1, True, seed=9)
    clk = torch.zeros(R * SLOTS * 4, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    L.damc_clock_probe(clk.data_ptr(), R * SLOTS)
    lv.posterior_langevin(z, x, G, E, 1, sigma, 0.1, True, seed=9)
    torch.cuda.synchronize()
    L.damc_clock_probe(None, 0)
    c = clk.view(R, SLOTS, 4).cpu().double()
    live = [c[r][c[r][:, 1] > 0] for r in range(R)]
    t0 = min(float(v[:, 1].min()) for v in live if len(v))
    print("== %s B=%d: one posterior step's limb-engine launches (us from the first workgroup start; 100 MHz)" % (net, B))
    for r, v in enumerate(live):
        if not len(v):
            continue
        st, en = (v[:, 1] - t0) / 100.0, (v[:, 3] - t0) / 100.0
        du = en - st
        ghz = ((v[:, 2] - v[:, 0]) / (v[:, 3] - v[:, 1]) / 10.0).median()  # shader clocks per 100 MHz tick
        print("launch %d: %4d workgroups  start q0/50/100 %s  end %s  per-WG %s us  clock %.2f GHz" % (
            r, len(v), [round(float(a), 1) for a in torch.quantile(st, q)],
            [round(float(a), 1) for a in torch.quantile(en, q)], [round(float(a), 1) for a in torch.quantile(du, q)],
            float(ghz)), flush=True)
    del G, E, x, z
    torch.cuda.empty_cache()
