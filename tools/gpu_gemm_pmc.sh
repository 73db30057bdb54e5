# MFMA-busy / wait PMC pass over the bench's limb-engine kernels (one bench block), reduced per kernel
export TMPDIR=/tmp
mkdir -p gpurun_out/gemm_pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY -d gpurun_out/gemm_pmc/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/gemm_pmc/pmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/gemm_pmc/pmc/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
seen = set()
for r in rows:
    k = r["Kernel_Name"]
    if "gemm_x3_kernel" not in k:
        continue
    key = k.split("(")[0]
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    did = r.get("Dispatch_Id") or r.get("Correlation_Id")
    if (key, did) not in seen:
        seen.add((key, did))
        cnt[key] += 1
for k, v in agg.items():
    gui = v["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
    busy = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * gui) if gui else 0
    wc = v["SQ_WAVE_CYCLES"]
    print("%-45s dispatches %3d  MFMA busy %.3f of SIMD-cycles  wait_any %.3f  wait_inst_lds %.3f  active_inst %.3f"
          % (k, cnt[k], busy, v["SQ_WAIT_ANY"] / wc if wc else 0, v["SQ_WAIT_INST_LDS"] / wc if wc else 0,
             v["SQ_ACTIVE_INST_ANY"] / wc if wc else 0))
PY
