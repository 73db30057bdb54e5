export TMPDIR=/tmp
timeout -k 10 200 ./tools/chain_probe 128 | head -3
timeout -k 10 600 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_ops.py tests/test_gpu_checkpoint.py -q -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_q.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/gpu_tests_q.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep_profile.py 128 2>&1 | grep -v amdgpu.ids
