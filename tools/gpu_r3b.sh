export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 180 tools/gemm_bench 128 > gpurun_out/r3b/gemm_pf.txt 2>&1 || exit 1
tail -8 gpurun_out/r3b/gemm_pf.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_graph.py tests/test_gpu_amortizer.py tests/test_gpu_dist.py tests/test_gpu_fid.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3b/tests.log; exit $rc
