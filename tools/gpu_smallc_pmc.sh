# PMC pass over tools/smallc_bench: where the output-layer dgrad kernels spend their wave cycles
export TMPDIR=/tmp
mkdir -p gpurun_out/scpmc
timeout -s KILL 90 rocprofv3 --kernel-trace -d gpurun_out/scpmc/trace -o run --output-format csv -- ./tools/smallc_bench > gpurun_out/scpmc/trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR -d gpurun_out/scpmc/pmc -o run --output-format csv -- ./tools/smallc_bench > gpurun_out/scpmc/pmc.log 2>&1 || { tail -5 gpurun_out/scpmc/pmc.log; exit 1; }
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open("gpurun_out/scpmc/pmc/run_counter_collection.csv")):
    k = r["Kernel_Name"][:70]
    if "dgrad" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
res = {}
for r in csv.DictReader(open("gpurun_out/scpmc/trace/run_kernel_trace.csv")):
    k = r["Kernel_Name"][:70]
    if "dgrad" in k: res[k] = (r.get("VGPR_Count") or r.get("Arch_VGPR_Count"), r.get("LDS_Block_Size"), r.get("Workgroup_Size"), r.get("Grid_Size"))
for k, d in agg.items():
    n = cnt[(k, "SQ_WAVES")]
    print(k, res.get(k))
    print("   " + "  ".join("%s=%.3g" % (c, v / max(1, cnt[(k, c)])) for c, v in sorted(d.items())))
PY
