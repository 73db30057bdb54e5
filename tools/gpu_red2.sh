# wave-per-tile split-K reduce: parity (split / shard bitwise tests, configs), then the reduce A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_langevin.py tests/test_gpu_ops.py tests/test_gpu_training.py -x -v --timeout 250 --timeout-method thread > gpurun_out/red_tests.log 2>&1
rc=$?; tail -3 gpurun_out/red_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_red_ab.sh
