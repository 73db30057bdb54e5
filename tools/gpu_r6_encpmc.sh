# round 6: FETCH_SIZE / WRITE_SIZE of one CelebA-HQ B=64 encoder call (is the encoder conv L2-miss bound?)
export TMPDIR=/tmp
O=gpurun_out/${1:-r6i}; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 64 1 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 64 1 > $O/write.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for c in ("fetch", "write"):
    f = glob.glob("gpurun_out/r6i/%s/**/*counter_collection.csv" % c, recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f))]
    rows = [r for r in rows if "gemm_x3_kernel" in r["Kernel_Name"] or "conv3" in r["Kernel_Name"]]
    for r in rows[-12:]:
        print(c, r["Kernel_Name"][:60], r["Counter_Name"], "%.1f MB" % (float(r["Counter_Value"]) * 1024 / 1e6))
PY
