# the CIFAR-10 encoder (nif 64, B=128) under rocprofv3: its kernels
export TMPDIR=/tmp
mkdir -p gpurun_out/enc
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/enc/trace -o run --output-format csv -- python3 tools/encoder_profile.py cifar10 128 10 > gpurun_out/enc/log.txt 2>&1 || exit 1
grep "per call" gpurun_out/enc/log.txt
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/enc/trace/run_kernel_stats.csv")))
for r in rows[:14]:
    print("%-70s %5s %9.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
