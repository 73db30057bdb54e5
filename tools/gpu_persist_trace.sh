# one traced persistent sweep (B=128 CIFAR Q) and its per-stage breakdown
export TMPDIR=/tmp
mkdir -p gpurun_out
DAMC_SWEEP_PERSIST=1 DAMC_SWEEP_TRACE=gpurun_out/sweep_trace.bin timeout -k 5 120 python3 tools/sweep_profile.py 128 > gpurun_out/ptrace.log 2>&1 || exit 1
python3 tools/sweep_trace.py gpurun_out/sweep_trace.bin
