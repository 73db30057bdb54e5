# round 6 checkpoint: every GPU test, then the default bench line
export TMPDIR=/tmp
O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 3000 $O/bench.json
