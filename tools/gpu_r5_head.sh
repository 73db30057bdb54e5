# round 5: the encoder's dense head -- its tests, then encoder wall time with the head on / off (interleaved), then a
# kernel-trace profile of the encoder with the head on
export TMPDIR=/tmp
O=gpurun_out/${1:-r5h}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_training.py tests/test_gpu_amortizer.py -m gpu -x -v \
  --timeout 120 --timeout-method thread -k "encoder" > $O/head_tests.log 2>&1
rc=$?; tail -3 $O/head_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for h in 1 0; do
    DAMC_ENC_HEAD=$h timeout -k 10 120 python tools/encoder_profile.py cifar10 128 20 > $O/enc_h$h.$r.txt 2>&1 || exit 1
    echo "head=$h $(cat $O/enc_h$h.$r.txt)"
  done
done | tee $O/head_ab.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o enc --output-format csv -- python3 tools/encoder_profile.py cifar10 128 20 \
  > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/encoder_kernel_stats.csv \;
head -14 $O/encoder_kernel_stats.csv
