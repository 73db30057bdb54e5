# round 6: reverse-sweep per-workgroup timeline (task start / wake / reduced / published), default and DBG=78
export TMPDIR=/tmp
O=gpurun_out/${1:-r6p}; mkdir -p $O
for d in 0 78; do
  DAMC_SWEEP_DBG=$d DAMC_SWEEP_TRACE=$O/trace_d$d.bin timeout -k 10 120 python tools/sweep_profile.py 128 > $O/prof_d$d.log 2>&1 || exit 1
  python3 tools/sweep_timeline.py $O/trace_d$d.bin > $O/timeline_d$d.txt || exit 1
  echo "== DBG=$d B=128"; cat $O/timeline_d$d.txt
done
