# channel-major K walk (variant 269) vs the default: GPU parity tests on the alternative build, then the bench A/B
export TMPDIR=/tmp
ALT=diffusion-amortized-mcmc_amd/damc/libdamc_cmaj.so
DAMC_LIB_PATH=$ALT timeout -k 10 400 python -u -m pytest tests/test_gpu_langevin.py tests/test_gpu_training.py tests/test_gpu_ops.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cmaj_tests.log 2>&1
rc=$?; tail -3 gpurun_out/cmaj_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_bench.sh $ALT
