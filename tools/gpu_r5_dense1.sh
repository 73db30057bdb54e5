# round 5: the first layer above the skinny rows on x3_dense_kernel -- bitwise tests, then the posterior step A/B and
# a kernel profile at B=128
export TMPDIR=/tmp
O=gpurun_out/${1:-r5d1}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_langevin.py tests/test_gpu_training.py -m gpu -x -v --timeout 150 \
  --timeout-method thread -k "skinny or split_k or f32a or sharded or full_width or g_update or generator" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/post_step_ab.py DAMC_X3_SKINNY 1,0 128 64 2>/dev/null | tee $O/dense1_ab.txt || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o ps --output-format csv -- \
  python3 tools/post_step_ab.py DAMC_X3_SKINNY 1 128 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/post_kernel_stats.csv \;
cut -c1-140 $O/post_kernel_stats.csv | head -12
