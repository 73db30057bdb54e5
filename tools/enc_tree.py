"""Encoder_* forward time of one library tree (argv[1]: a checkout holding diffusion-amortized-mcmc_amd/ with its own
built libdamc.so), net:B cases after it; median of 5 samples of three back-to-back calls, and an xemb checksum."""
import hashlib
import os
import sys

tree = os.path.abspath(sys.argv[1])
sys.path[:0] = [os.path.join(tree, "diffusion-amortized-mcmc_amd")]
import torch  # noqa: E402

from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

dev = torch.device("cuda:0")
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for case in sys.argv[2:]:
    name, B = case.split(":")[0], int(case.split(":")[1])
    hw = {"cifar10": 32, "celeba64": 64, "celebaHQ": 256}[name]
    enc = synth.load_into(getattr(dn, "Encoder_" + name)(nc=3, nemb=1024, nif=64), 3).to(dev).eval()
    x = torch.from_numpy(synth.uniform_f32(13, 1, (B, 3, hw, hw))).to(dev)
    out = amortizer.encoder_forward(enc, x)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        a.record()
        for _ in range(3):
            amortizer.encoder_forward(enc, x)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / 3)
    print("%s %s B=%d %.4f ms per call, xemb %s" % (os.path.basename(tree), name, B, sorted(ts)[2],
                                                     hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]),
          flush=True)
