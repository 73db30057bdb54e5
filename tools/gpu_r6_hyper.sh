# round 6: the sweep's hyper GEMMs on the 64 x 256 tile (hyper2_x3_kernel) vs round 5's 128 x 64 (DAMC_SWEEP_HYPER=v1)
export TMPDIR=/tmp
O=gpurun_out/${1:-r6y}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_amortizer.py > $O/tests.txt 2>&1; tail -1 $O/tests.txt
for b in 128 8; do
  timeout -k 10 180 python tools/sweep_ab.py $b DAMC_SWEEP_HYPER=limb DAMC_SWEEP_HYPER=v1 > $O/hyper_ab_b$b.txt 2>&1 || exit 1
  grep sweep $O/hyper_ab_b$b.txt
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/sweep -o run --output-format csv -- python3 tools/sweep_profile.py 128 > $O/sweep.log 2>&1 || exit 1
python3 tools/kstats.py $(find $O/sweep -name '*kernel_stats.csv' | head -1) 6
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 tools/sweep_profile.py 128 > $O/fetch.log 2>&1 || exit 1
O=$O python3 - <<'PY'
import csv, glob, collections, os
f = glob.glob(os.environ["O"] + "/fetch/**/*counter_collection.csv", recursive=True)[0]
acc, n = collections.defaultdict(float), collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    if "hyper" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:50]] += float(r["Counter_Value"]); n[r["Kernel_Name"][:50]].add(r["Dispatch_Id"])
for k in acc:
    print("FETCH_SIZE %s: %.1f MB per dispatch (x2: %.1f MB)" % (k, acc[k] / len(n[k]) / 1024, 2 * acc[k] / len(n[k]) / 1024))
PY
