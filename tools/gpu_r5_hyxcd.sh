# round 5: XCD-grouped tile order of the sweep's hyper GEMMs -- sweep tests, then the A/B
export TMPDIR=/tmp
O=gpurun_out/${1:-r5hx}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_amortizer.py -m gpu -x -v --timeout 150 --timeout-method thread \
  -k "sweep or hyper" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/sweep_hyper_ab.py 3 DAMC_SWEEP_HYPER_XCD=1,DAMC_SWEEP_HYPER_XCD=0 2>/dev/null | tee $O/hyxcd_ab.txt || exit 1
