export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
timeout -k 10 300 python tools/diag_team_capture.py > gpurun_out/r3c/diag_team_capture.txt 2>&1 || exit 1
cat gpurun_out/r3c/diag_team_capture.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3c/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3c/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err || exit 1
tail -c 300 gpurun_out/r3c/bench.json
