# round 6: encoder host submission time vs GPU time (CIFAR B=128, HQ B=8 / 64), then HQ B=8 and CIFAR dispatches
export TMPDIR=/tmp
O=gpurun_out/${1:-r6t}; mkdir -p $O
for cfg in "cifar10 128" "celebaHQ 8" "celebaHQ 64"; do
  set -- $cfg
  timeout -k 10 120 python tools/enc_hosttime.py $1 $2 30 > $O/host_$1_$2.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/host_$1_$2.txt
done
for cfg in "celebaHQ 8" "cifar10 128"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc_$1_$2 -o run --output-format csv -- python3 tools/encoder_profile.py $1 $2 3 > $O/enc_$1_$2.log 2>&1 || exit 1
  f=$(find $O/enc_$1_$2 -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_tail.py $f "conv3_|pack_conv_x3_lds|enc_first" "$1 encoder B=$2: one call" > $O/enc_$1_$2_dispatches.txt || exit 1
  cat $O/enc_$1_$2_dispatches.txt
done
