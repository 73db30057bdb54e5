# output-layer dgrad on the limb engine: A/B vs the VALU kernel, the Langevin / config parity tests, a short bench
export TMPDIR=/tmp
mkdir -p gpurun_out
# (limb GEMM A/B: tools/gpu_gemm_clock.sh)
timeout -k 10 120 ./tools/smallc_bench > gpurun_out/smallc2.txt 2>&1; rc=$?; cat gpurun_out/smallc2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_langevin.py tests/test_gpu_configs.py tests/test_gpu_dropin.py tests/test_gpu_checkpoint.py -x -v --timeout 200 --timeout-method thread > gpurun_out/lv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/bench_smallc.json 2> gpurun_out/bench_smallc.err || exit 1
tail -c 700 gpurun_out/bench_smallc.json
