# round 6: sweep_fast_kernel refinements (compile-time load counts, z image writes spread over the waves, pad zeroed
# once): amortizer tests, then the A/B against the generic kernel and the per-stage trace
export TMPDIR=/tmp
O=gpurun_out/${1:-r6w}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_amortizer.py > $O/tests.txt 2>&1; tail -1 $O/tests.txt
for b in 128 8; do
  timeout -k 10 180 python tools/sweep_ab.py $b DAMC_SWEEP_FAST=1 DAMC_SWEEP_FAST=0 > $O/fast_ab_b$b.txt 2>&1 || exit 1
  grep sweep $O/fast_ab_b$b.txt
done
DAMC_SWEEP_TRACE=$O/trace_fast.bin timeout -k 10 120 python tools/sweep_profile.py 128 > $O/prof_fast.log 2>&1 || exit 1
python3 tools/sweep_trace.py $O/trace_fast.bin | tee $O/trace_fast.txt
