# per-stage timeline of the team sweep (DAMC_SWEEP_TRACE stamps) under the default sentinel protocol and the probes
export TMPDIR=/tmp
mkdir -p gpurun_out/strace
for d in 0 2 4 16; do
  echo "== DAMC_SWEEP_DBG=$d"
  DAMC_SWEEP_DBG=$d timeout -k 10 120 python tools/sweep_trace_dbg.py gpurun_out/strace/t$d.bin 2>&1 | grep -v "amdgpu.ids\|Conditional" || exit 1
done
