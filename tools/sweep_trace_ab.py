"""Stage traces (DAMC_SWEEP_TRACE) of the team sweep at B=128 for the drained-flag and the sentinel hand-off, one
process; then tools/sweep_trace.py on each dump."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.makedirs(os.path.join(HERE, "gpurun_out"), exist_ok=True)
os.environ["DAMC_SWEEP_TRACE"] = os.path.join(HERE, "gpurun_out", "trace_warm.bin")
sys.path[:0] = [os.path.join(HERE, "diffusion-amortized-mcmc_amd"), HERE]
import torch  # noqa: E402

from damc import amortizer, synth  # noqa: E402
from src import diffusion_net as dn  # noqa: E402

dev = torch.device("cuda:0")
Q = dn._netQ_U(nc=3, nz=128, nxemb=1024, ntemb=128, nif=64, diffusion_residual=True, n_interval=100, logsnr_min=-5.1,
               logsnr_max=9.8, var_type="large", with_noise=True, dataset="cifar10")
synth.load_into(Q, 20)
Q.to(dev).eval()
xemb = torch.from_numpy(synth.normal_f32(7, 0, (128, 1024))).to(dev)
zt0 = torch.from_numpy(synth.normal_f32(8, 0, (128, 128))).to(dev)
for sent in ("0", "1", "0", "1"):
    os.environ["DAMC_SWEEP_SENT"] = sent
    f = os.path.join(HERE, "gpurun_out", "trace_sent%s.bin" % sent)
    os.environ["DAMC_SWEEP_TRACE"] = f
    z = zt0.clone()
    amortizer.reverse_sweep(Q, xemb, z, seed=11)
    torch.cuda.synchronize()
for sent in ("0", "1"):
    print("== DAMC_SWEEP_SENT=%s" % sent, flush=True)
    subprocess.check_call([sys.executable, os.path.join(HERE, "tools", "sweep_trace.py"),
                           os.path.join(HERE, "gpurun_out", "trace_sent%s.bin" % sent)])
