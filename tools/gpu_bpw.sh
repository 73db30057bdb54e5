# split-K register slab layout vs row-major: parity (the split / shard bitwise tests and the configs) and the per-rank legs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_langevin.py tests/test_gpu_ops.py tests/test_gpu_training.py -x -v --timeout 250 --timeout-method thread > gpurun_out/bpw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bpw_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 0 1; do
  if [ $b = 0 ]; then export DAMC_X3_KSLAB_REG=0; else unset DAMC_X3_KSLAB_REG; fi
  echo "== register slab layout: $b"
  timeout -k 10 120 python3 tools/b16_profile.py 16 2>&1 | grep "per posterior" || exit 1
  timeout -k 10 120 python3 tools/b16_profile.py 8 2>&1 | grep "per posterior" || exit 1
  timeout -k 10 120 python3 tools/b16_profile.py 32 2>&1 | grep "per posterior" || exit 1
done
timeout -k 10 300 python3 bench.py > gpurun_out/bpw_bench.json 2> gpurun_out/bpw_bench.err && cat gpurun_out/bpw_bench.json
