# the strong-scaling per-rank batch (CIFAR B=16) under rocprofv3: which kernels bound it
export TMPDIR=/tmp
mkdir -p gpurun_out/b16
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/b16/trace -o run --output-format csv -- python3 tools/b16_profile.py 16 > gpurun_out/b16/log.txt 2>&1 || exit 1
grep "per posterior" gpurun_out/b16/log.txt
head -16 gpurun_out/b16/trace/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
