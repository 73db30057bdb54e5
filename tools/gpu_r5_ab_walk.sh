# round 5: the F32A limb GEMM with the supertile raster (V 277 = 261 | 16) and the channel-major K walk (V 269 = 261 | 8)
# against the default (261), same box, interleaved; then FETCH_SIZE and kernel times per variant
export TMPDIR=/tmp
O=gpurun_out/${1:-r5j}; mkdir -p $O
for r in 1 2 3; do
  for t in . tools/ab/v277 tools/ab/v269; do
    timeout -k 5 120 python3 tools/cfg_versions.py $t cifar128 cifar16 >> $O/walk_ab.txt 2>&1 || exit 1
  done
done
cat $O/walk_ab.txt
for t in . tools/ab/v277 tools/ab/v269; do
  n=$(basename $t)
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_$n -o run --output-format csv -- python3 tools/cfg_versions.py $t cifar128 > /dev/null 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$n -o run --output-format csv -- python3 tools/cfg_versions.py $t cifar128 > /dev/null 2>&1 || exit 1
done
