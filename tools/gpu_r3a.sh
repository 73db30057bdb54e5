# round 3 first refresh: GEMM timing probes, GPU tests (incl. launcher / dist / rescue / team-capture tests), bench
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 180 tools/gemm_bench 128 > gpurun_out/r3a/gemm_probe.txt 2>&1 || exit 1
tail -8 gpurun_out/r3a/gemm_probe.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3a/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3a/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err || exit 1
tail -c 400 gpurun_out/r3a/bench.json
