# round 5: split-K reduces with batched slab loads -- bitwise tests, then posterior steps at the per-rank / headline
# batches against the HEAD build (tools/ab/base, DAMC_LIB_PATH), interleaved
export TMPDIR=/tmp
O=gpurun_out/${1:-r5rd}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_langevin.py tests/test_gpu_dist.py -m gpu -x -v --timeout 150 \
  --timeout-method thread -k "split_k or sharded or f32a or skinny or fused or bitwise or chunk" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export DAMC_LIB_PATH=$PWD/tools/ab/base/diffusion-amortized-mcmc_amd/damc/libdamc.so; else unset DAMC_LIB_PATH; fi
    timeout -k 10 200 python tools/post_step_ab.py DAMC_NOOP $lib 16 32 128 2>/dev/null || exit 1
  done
done | tee $O/reduce_ab.txt
