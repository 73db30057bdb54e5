# round 5: x3_skinny_kernel with 32 columns per wave (DAMC_X3_SKINNY_NTW=2) -- bitwise test, then the per-rank step A/B
export TMPDIR=/tmp
O=gpurun_out/${1:-r5nt}; mkdir -p $O
DAMC_X3_SKINNY_NTW=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_langevin.py -m gpu -x -v --timeout 150 \
  --timeout-method thread -k "skinny" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/post_step_ab.py DAMC_X3_SKINNY_NTW 1,2 16 32 2>/dev/null | tee $O/ntw_ab.txt || exit 1
timeout -k 10 300 python tools/post_step_ab.py DAMC_X3_SKINNY_NTW 1,2 16 32 2>/dev/null | tee -a $O/ntw_ab.txt || exit 1
