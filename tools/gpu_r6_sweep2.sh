# round 6: reverse-sweep team kernel with parts switched off (DAMC_SWEEP_DBG, timing only: wrong results), B=128
export TMPDIR=/tmp
O=gpurun_out/${1:-r6o}; mkdir -p $O
for d in 0 2 66 8 74 4 78; do
  DAMC_SWEEP_DBG=$d DAMC_SWEEP_TRACE=$O/trace_d$d.bin timeout -k 10 120 python tools/sweep_profile.py 128 > $O/prof_d$d.log 2>&1 || exit 1
  python3 tools/sweep_trace.py $O/trace_d$d.bin > $O/sweep_trace_d$d.txt || exit 1
  echo "== DBG=$d B=128"; cat $O/sweep_trace_d$d.txt; grep denoise_chain $O/prof_d$d.log
done
