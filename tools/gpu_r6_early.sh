# round 6: team sweep with the handed-off loads issued at task start (DAMC_SWEEP_EARLY=1) vs after the setup (0)
export TMPDIR=/tmp
O=gpurun_out/${1:-r6q}; mkdir -p $O
for b in 128 8; do
  timeout -k 10 180 python tools/sweep_ab.py $b DAMC_SWEEP_EARLY=1 DAMC_SWEEP_EARLY=0 > $O/early_ab_b$b.txt 2>&1 || exit 1
  cat $O/early_ab_b$b.txt
done
for e in 1 0; do
  DAMC_SWEEP_EARLY=$e DAMC_SWEEP_TRACE=$O/trace_e$e.bin timeout -k 10 120 python tools/sweep_profile.py 128 > $O/prof_e$e.log 2>&1 || exit 1
  python3 tools/sweep_timeline.py $O/trace_e$e.bin > $O/timeline_e$e.txt || exit 1
  python3 tools/sweep_trace.py $O/trace_e$e.bin > $O/trace_e$e.txt || exit 1
  echo "== EARLY=$e"; head -12 $O/timeline_e$e.txt; cat $O/trace_e$e.txt
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_amortizer.py -k "team or rescue or deterministic or golden" > $O/tests.txt 2>&1; tail -3 $O/tests.txt
