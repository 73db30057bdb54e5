export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_langevin.py tests/test_gpu_ops.py -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ct.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_ct.log
[ $rc -eq 0 ] || exit $rc
for d in 0 31; do
  DAMC_CHAIN_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ct$d -o run --output-format csv -- python3 tools/sweep_profile.py 128 > gpurun_out/ct$d.log 2>&1 || exit 1
  echo "dbg=$d"; grep -o "'us_per_denoise_step': [0-9.]*" gpurun_out/ct$d.log; python3 tools/chain_trace.py $(find gpurun_out/ct$d -name "*kernel_trace.csv" | head -1)
done
timeout -k 10 300 python tools/ebm_profile.py
