# split-K reduce changes: parity (split / shard bitwise tests, configs) then per-rank step timings
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_langevin.py tests/test_gpu_ops.py tests/test_gpu_training.py -x -v --timeout 250 --timeout-method thread > gpurun_out/red_tests.log 2>&1
rc=$?; tail -3 gpurun_out/red_tests.log; [ $rc -eq 0 ] || exit $rc
for B in 8 16 32; do timeout -k 10 120 python3 tools/b16_profile.py $B 2>&1 | grep "per posterior" || exit 1; done
timeout -k 10 200 python3 tools/cfg_profile.py _netG_celebaHQ 128 128 256 8 3 2>&1 | grep "per posterior" || exit 1
timeout -k 10 200 python3 tools/cfg_profile.py _netG_celeba64 128 128 64 32 5 2>&1 | grep "per posterior" || exit 1
