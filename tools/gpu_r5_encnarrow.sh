# round 5: CIFAR B=128 encoder over DAMC_ENC_F32A x DAMC_X3_NARROW (the 64 x 128 tile unsplit where it fills the chip),
# interleaved twice
export TMPDIR=/tmp
O=gpurun_out/${1:-r5en}; mkdir -p $O
for r in 1 2; do
  for f in 1 0; do
    for nw in 0 1; do
      DAMC_ENC_F32A=$f DAMC_X3_NARROW=$nw timeout -k 10 120 python tools/encoder_profile.py cifar10 128 20 > $O/e.txt 2>/dev/null || exit 1
      echo "f32a=$f narrow=$nw $(cat $O/e.txt)"
    done
  done
done | tee $O/enc_narrow_ab.txt
