# round 5: the encoder norms' slab sums with two slabs in flight -- encoder tests, then the CIFAR B=128 encoder against
# the HEAD build (tools/ab/base, DAMC_LIB_PATH), interleaved
export TMPDIR=/tmp
O=gpurun_out/${1:-r5is}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_amortizer.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "encoder" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for lib in new base; do
    if [ $lib = base ]; then export DAMC_LIB_PATH=$PWD/tools/ab/base/diffusion-amortized-mcmc_amd/damc/libdamc.so; else unset DAMC_LIB_PATH; fi
    timeout -k 10 120 python tools/encoder_profile.py cifar10 128 20 > $O/e.txt 2>/dev/null || exit 1
    echo "$lib $(cat $O/e.txt)"
  done
done | tee $O/inslab_ab.txt
