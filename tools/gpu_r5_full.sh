# round 5 full refresh: every GPU test, the default bench line, then tools/profile_round.sh's passes
export TMPDIR=/tmp
O=gpurun_out/${1:-r5k}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 400 $O/bench.json
bash tools/profile_round.sh $O/prof || exit 1
timeout -k 10 300 python3 tools/train_iter_profile.py --damc-optim > $O/train_iter.txt 2>&1 || exit 1
