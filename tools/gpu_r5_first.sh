# round 5: the two-pass first layer's statistics pass over 4-pixel runs -- encoder tests, then CelebA-HQ encoder time
# over DAMC_ENC_FIRST_PX (interleaved) and a profile
export TMPDIR=/tmp
O=gpurun_out/${1:-r5fp}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_amortizer.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -k "encoder" > $O/enc_tests.log 2>&1
rc=$?; tail -3 $O/enc_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 4 1; do
    for B in 64 8; do
      DAMC_ENC_FIRST_PX=$f timeout -k 10 120 python tools/encoder_profile.py celebaHQ $B 10 > $O/e.txt 2>/dev/null || exit 1
      echo "first_px=$f $(cat $O/e.txt)"
    done
  done
done | tee $O/hq_first_px_ab.txt
bash tools/gpu_r5_hqenc.sh ${1:-r5fp}
