# round 5: F32A after the big-image norms -- encoder tests, then CelebA-HQ encoder time over DAMC_ENC_F32A (interleaved)
export TMPDIR=/tmp
O=gpurun_out/${1:-r5hf}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_amortizer.py tests/test_gpu_checkpoint.py \
  -m gpu -x -v --timeout 120 --timeout-method thread -k "encoder or checkpoint" > $O/enc_tests.log 2>&1
rc=$?; tail -3 $O/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 1 0; do
    for B in 64 8; do
      DAMC_ENC_F32A=$f timeout -k 10 120 python tools/encoder_profile.py celebaHQ $B 10 > $O/e.txt 2>/dev/null || exit 1
      echo "f32a=$f $(cat $O/e.txt)"
    done
  done
done | tee $O/hq_f32a_ab.txt
timeout -k 10 120 python tools/enc_hosttime.py cifar10 128 50 2>/dev/null | tee $O/enc_hosttime.txt || exit 1
bash tools/gpu_r5_hqenc.sh ${1:-r5hf}
