export TMPDIR=/tmp
mkdir -p gpurun_out/encprof2
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_amortizer.py -k "encoder or q_sweep or dropin" -v -s --timeout 300 --timeout-method thread > gpurun_out/encprof2/tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/encprof2/tests.log | tail -1; grep -E "xemb" gpurun_out/encprof2/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/encprof2/c -o run --output-format csv -- python3 tools/encoder_profile.py cifar10 128 5 > gpurun_out/encprof2/c.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/encprof2/h -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 64 3 > gpurun_out/encprof2/h.log 2>&1 || exit 1
grep "per call" gpurun_out/encprof2/c.log gpurun_out/encprof2/h.log
