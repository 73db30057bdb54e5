# round 5: the dense head's tests, then encoder wall time over DAMC_ENC_HEAD / DAMC_ENC_HEAD_PD (interleaved), then a
# kernel-trace profile of the encoder
export TMPDIR=/tmp
O=gpurun_out/${1:-r5h2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_training.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "dense_head or one_call" > $O/head_tests.log 2>&1
rc=$?; tail -3 $O/head_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "1 4 1" "1 4 0" "1 1 1" "0 4 1"; do
    set -- $v
    DAMC_ENC_HEAD=$1 DAMC_ENC_HEAD_PD=$2 DAMC_ENC_HEAD_XCD=$3 timeout -k 10 120 python tools/encoder_profile.py cifar10 128 20 \
      > $O/enc.txt 2>/dev/null || exit 1
    echo "head=$1 pd=$2 xcd=$3 $(cat $O/enc.txt)"
  done
done | tee $O/head_ab.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o enc --output-format csv -- \
  python3 tools/encoder_profile.py cifar10 128 20 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/encoder_kernel_stats.csv \;
cut -c1-150 $O/encoder_kernel_stats.csv
