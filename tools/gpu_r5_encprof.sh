# round 5: kernel-trace profile of the CIFAR B=128 encoder (dense head on) and the Q update
export TMPDIR=/tmp
O=gpurun_out/${1:-r5e}; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o enc --output-format csv -- \
  python3 tools/encoder_profile.py cifar10 128 20 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/encoder_kernel_stats.csv \;
cat $O/encoder_kernel_stats.csv | cut -c1-200
