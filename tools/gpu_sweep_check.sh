set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_ops.py tests/test_gpu_checkpoint.py tests/test_gpu_dropin.py -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1
rc=$?
tail -6 gpurun_out/gpu_tests3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sweep_profile.py 128 > gpurun_out/sweep_graph.txt 2>&1 && cat gpurun_out/sweep_graph.txt | tail -2
DAMC_SWEEP_GRAPH=0 timeout -k 10 300 python tools/sweep_profile.py 128 > gpurun_out/sweep_nograph.txt 2>&1 && tail -1 gpurun_out/sweep_nograph.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sweep_prof -o run --output-format csv -- python3 tools/sweep_profile.py 128 > gpurun_out/sweep_prof.log 2>&1
find gpurun_out/sweep_prof -name "*kernel_stats.csv" | head -1 | xargs head -12
