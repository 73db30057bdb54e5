# round 6: reverse-sweep per-stage trace (team kernel) at B=128 and B=8, and the in0 probes (wrong results, timing only)
export TMPDIR=/tmp
O=gpurun_out/${1:-r6n}; mkdir -p $O
for b in 128 8; do
  DAMC_SWEEP_TRACE=$O/trace$b.bin timeout -k 10 120 python tools/sweep_profile.py $b > $O/prof$b.log 2>&1 || exit 1
  python3 tools/sweep_trace.py $O/trace$b.bin > $O/sweep_trace_b$b.txt || exit 1
  echo "== B=$b"; cat $O/sweep_trace_b$b.txt; grep -E "us_per|launches" $O/prof$b.log
done
for d in 32 64 96; do
  DAMC_SWEEP_DBG=$d DAMC_SWEEP_TRACE=$O/trace_d$d.bin timeout -k 10 120 python tools/sweep_profile.py 128 > $O/prof_d$d.log 2>&1 || exit 1
  python3 tools/sweep_trace.py $O/trace_d$d.bin > $O/sweep_trace_d$d.txt || exit 1
  echo "== DBG=$d B=128"; cat $O/sweep_trace_d$d.txt
done
