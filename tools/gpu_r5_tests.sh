# every GPU test (round 5), log under gpurun_out/<tag>
export TMPDIR=/tmp
O=gpurun_out/${1:-r5n}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; exit $rc
