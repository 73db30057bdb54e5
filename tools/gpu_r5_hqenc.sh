# round 5: kernel-trace profile of the CelebA-HQ encoder at B=64 (config 5's one-GPU batch) and B=8
export TMPDIR=/tmp
O=gpurun_out/${1:-r5q}; mkdir -p $O
for B in 64 8; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof$B -o enc --output-format csv -- \
    python3 tools/encoder_profile.py celebaHQ $B 5 > $O/prof$B.log 2>&1 || exit 1
  find $O/prof$B -name "*kernel_stats.csv" -exec cp {} $O/hq_b${B}_kernel_stats.csv \;
  grep "encoder" $O/prof$B.log
  cut -c1-170 $O/hq_b${B}_kernel_stats.csv | head -16
done
