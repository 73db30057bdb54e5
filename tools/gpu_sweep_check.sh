# reverse sweep: amortizer + config parity tests, then us per denoise step and the per-class split
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_configs.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sweep_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python3 tools/sweep_profile.py 128
