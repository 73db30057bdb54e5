# k4 s2 output-layer dgrad with wave-uniform pixels (scalar delta loads): parity, then A/B (DAMC_SMALLC_UNI)
export TMPDIR=/tmp
mkdir -p gpurun_out
DAMC_SMALLC_UNI=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_langevin.py tests/test_gpu_ops.py tests/test_gpu_training.py -x -v --timeout 250 --timeout-method thread > gpurun_out/uni_tests.log 2>&1
rc=$?; tail -2 gpurun_out/uni_tests.log; [ $rc -eq 0 ] || exit $rc
for u in 0 1 0 1; do
  export DAMC_SMALLC_UNI=$u
  echo "== uniform-pixel dgrad $u"
  timeout -k 10 200 python3 tools/cfg_profile.py _netG_celebaHQ 128 128 256 8 3 2>&1 | grep "per posterior" || exit 1
  timeout -k 10 200 python3 tools/cfg_profile.py _netG_svhn 100 64 32 64 5 2>&1 | grep "per posterior" || exit 1
  timeout -k 10 200 python3 tools/cfg_profile.py _netG_celeba64 100 128 64 32 5 2>&1 | grep "per posterior" || exit 1
done
