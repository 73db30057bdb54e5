export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/sweep_profile.py 128 > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 tools/sweep_profile.py 128 > $O/write.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for kind in ("fetch", "write"):
    f = glob.glob("gpurun_out/r6x/%s/**/*counter_collection.csv" % kind, recursive=True)[0]
    acc, n = collections.defaultdict(float), collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        acc[k] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k in sorted(acc, key=lambda k: -acc[k])[:8]:
        print(kind, "%-60s %5d dispatches %10.1f MB per dispatch (raw counter, KB units x1024?)" % (k, len(n[k]), acc[k] / len(n[k]) / 1024))
PY
