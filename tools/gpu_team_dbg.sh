# team sweep per-stage trace for DAMC_SWEEP_DBG variants (timing only: dbg != 0 gives wrong results)
mkdir -p gpurun_out
for d in "$@"; do
  echo "== dbg=$d"
  DAMC_SWEEP_DBG=$d DAMC_SWEEP_TRACE=gpurun_out/team_trace_$d.bin timeout -k 5 120 python3 tools/sweep_profile.py 128 > gpurun_out/tt_$d.log 2>&1 || exit 1
  python3 tools/sweep_trace.py gpurun_out/team_trace_$d.bin
done
