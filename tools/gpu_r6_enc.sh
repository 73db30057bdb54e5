# round 6: one CelebA-HQ encoder call's dispatches at B=64 and B=8, and CIFAR B=128 (kernel trace)
export TMPDIR=/tmp
O=gpurun_out/${1:-r6h}; mkdir -p $O
for cfg in "celebaHQ 64" "celebaHQ 8" "cifar10 128"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc_$1_$2 -o run --output-format csv -- python3 tools/encoder_profile.py $1 $2 3 > $O/enc_$1_$2.log 2>&1 || exit 1
  f=$(find $O/enc_$1_$2 -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_tail.py $f "conv3_|pack_conv_x3_lds|enc_first" "$1 encoder B=$2: one call" > $O/enc_$1_$2_dispatches.txt || exit 1
  cat $O/enc_$1_$2_dispatches.txt; tail -1 $O/enc_$1_$2.log
done
