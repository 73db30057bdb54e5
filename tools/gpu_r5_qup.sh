# Q update round 5: training tests, then the update timed (A/B over the new paths), then a rocprof trace
export TMPDIR=/tmp
O=gpurun_out/${1:-r5d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_optim.py tests/test_gpu_amortizer.py -x -v --timeout 120 --timeout-method thread > $O/train_tests.log 2>&1
rc=$?; tail -3 $O/train_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "" "" ""; do
  echo "[$v] $(env $v timeout -k 5 60 python3 tools/q_update_trace.py 20 2>&1 | tail -1)" >> $O/qup_ab.txt || exit 1
done
cat $O/qup_ab.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/qup -o run --output-format csv -- python3 tools/q_update_trace.py 5 > $O/qup.log 2>&1 || exit 1
timeout -k 5 120 python3 tools/q_update_hosttime.py 50 > $O/hosttime.txt 2>&1 || exit 1
