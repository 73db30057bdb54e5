# round 5: the sweep's hyper GEMMs on the limb product -- sweep / amortizer / graph / config tests, the A/B, a profile
export TMPDIR=/tmp
O=gpurun_out/${1:-r5hy}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_graph.py tests/test_gpu_checkpoint.py \
  tests/test_gpu_configs.py -m gpu -x -v --timeout 150 --timeout-method thread -k "sweep or hyper or amortizer or graph or checkpoint or q_ or Q" \
  > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/sweep_hyper_ab.py 2 2>/dev/null | tee $O/sweep_hyper_ab.txt || exit 1
DAMC_SWEEP_HYPER=limb timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o sw --output-format csv -- \
  python3 tools/sweep_hyper_ab.py 1 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/sweep_kernel_stats.csv \;
cut -c1-150 $O/sweep_kernel_stats.csv | head -12
