# mean FETCH_SIZE (x2 gfx950 correction, bytes) per gemm_x3_kernel instantiation from a rocprofv3 --pmc run of
# tools/gemm_bench: usage gemm_fetch.py DIR
import csv, sys
from collections import defaultdict
tot, n = defaultdict(float), defaultdict(int)
for r in csv.DictReader(open(sys.argv[1] + "/run_counter_collection.csv")):
    k = r["Kernel_Name"]
    if "gemm_x3_kernel" not in k:
        continue
    key = k[k.index("gemm_x3_kernel"):].split("(")[0]
    tot[key] += float(r["Counter_Value"])
    n[key] += 1
for k in sorted(tot):
    print("%-40s launches %4d  FETCH %.3f GB per launch" % (k, n[k], 2 * tot[k] / n[k] * 1024 / 1e9))
