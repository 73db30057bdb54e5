"""Per-workgroup start / K-loop end of every limb-engine launch of one encoder call (damc_clock_probe stamps, 100 MHz
realtime; DAMC_CLOCK_REGIONS gives each launch its own slot region): how much of a conv's launch is its K loops, and
how much is the rest (prologue, epilogue, the gap between a CU's workgroups)?
usage: python tools/enc_wg_probe.py [net:B ...]   (default celebaHQ:64 celebaHQ:8 cifar10:128; run through gpurun)"""
import os
import sys

os.environ.setdefault("DAMC_CLOCK_REGIONS", "8")
import torch  # noqa: E402

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
from damc import _lib, amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

R, SLOTS = int(os.environ["DAMC_CLOCK_REGIONS"]), 4096
dev = torch.device("cuda:0")
L = _lib.lib()
q = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
ncu = torch.cuda.get_device_properties(dev).multi_processor_count
for case in (sys.argv[1:] or ["celebaHQ:64", "celebaHQ:8", "cifar10:128"]):
    name, B = case.split(":")[0], int(case.split(":")[1])
    hw = {"cifar10": 32, "celeba64": 64, "celebaHQ": 256}[name]
    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 1, (B, 3, hw, hw))).to(dev)
    for _ in range(3):
        amortizer.encoder_forward(enc, x)
    clk = torch.zeros(R * SLOTS * 4, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    L.damc_clock_probe(clk.data_ptr(), R * SLOTS)
    amortizer.encoder_forward(enc, x)
    torch.cuda.synchronize()
    L.damc_clock_probe(None, 0)
    c = clk.view(R, SLOTS, 4).cpu().double()
    live = [c[r][c[r][:, 1] > 0] for r in range(R)]
    print("== encoder %s B=%d: limb-engine launches (us from the launch's first workgroup start; 100 MHz; %d CUs)"
          % (name, B, ncu))
    for r, v in enumerate(live):
        if not len(v):
            continue
        t0 = float(v[:, 1].min())
        st, en = (v[:, 1] - t0) / 100.0, (v[:, 3] - t0) / 100.0
        du = en - st
        span = float(en.max())
        # K-loop share: the workgroups' K-loop time over the CU-time the launch spans (one workgroup per CU)
        share = float(du.sum()) / (span * min(ncu, len(v)))
        ghz = ((v[:, 2] - v[:, 0]) / (v[:, 3] - v[:, 1]) / 10.0).median()
        print("launch %d: %5d workgroups  span %.1f us  K-loop per WG q0/50/100 %s us  K-loop share %.2f  clock %.2f GHz"
              % (r, len(v), span, [round(float(a), 1) for a in torch.quantile(du, q)], share, float(ghz)), flush=True)
    del enc, x
    torch.cuda.empty_cache()
