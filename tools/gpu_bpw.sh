# multi-block split-K slices: parity (the split / shard bitwise tests and the configs) and the per-rank legs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_langevin.py tests/test_gpu_ops.py tests/test_gpu_training.py -x -v --timeout 250 --timeout-method thread > gpurun_out/bpw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bpw_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 1 0; do
  if [ $b = 1 ]; then export DAMC_X3_KSPLIT_BPW=1; else unset DAMC_X3_KSPLIT_BPW; fi
  echo "== bpw pinned to 1: $b"
  timeout -k 10 120 python3 tools/b16_profile.py 16 2>&1 | grep "per posterior" || exit 1
  timeout -k 10 120 python3 tools/b16_profile.py 8 2>&1 | grep "per posterior" || exit 1
  timeout -k 10 120 python3 tools/b16_profile.py 32 2>&1 | grep "per posterior" || exit 1
done
