export TMPDIR=/tmp
mkdir -p gpurun_out/tdbg
for d in 0 8 1 2; do
  echo "== DAMC_SWEEP_DBG=$d"
  DAMC_SWEEP_DBG=$d timeout -k 10 120 python tools/sweep_trace_dbg.py gpurun_out/tdbg/t$d.bin 2>&1 | grep -v "amdgpu.ids\|Conditional" || exit 1
done
