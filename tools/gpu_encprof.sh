export TMPDIR=/tmp
mkdir -p gpurun_out/encprof
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/encprof/c -o run --output-format csv -- python3 tools/encoder_profile.py cifar10 128 5 > gpurun_out/encprof/c.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/encprof/h -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 64 3 > gpurun_out/encprof/h.log 2>&1 || exit 1
grep "per call" gpurun_out/encprof/c.log gpurun_out/encprof/h.log
for d in c h; do f=$(find gpurun_out/encprof/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; head -14 $f | cut -d, -f1-5; done
