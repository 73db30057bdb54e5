# persistent reverse-sweep chain: amortizer parity tests and the sweep timing with DAMC_SWEEP_PERSIST=1
export TMPDIR=/tmp
mkdir -p gpurun_out
DAMC_SWEEP_PERSIST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_amortizer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/persist_tests.log 2>&1
rc=$?; tail -5 gpurun_out/persist_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  echo -n "persist=$v "; DAMC_SWEEP_PERSIST=$v timeout -k 5 120 python3 tools/sweep_profile.py 128 2>&1 | grep -o "'us_per_denoise_step': [0-9.]*\|denoise_chain.*" | tr '\n' ' ' || exit 1; echo
done
