# EBM MFMA evidence: parity, engine sweep, kernel trace and MFMA-busy PMC passes at B = 16384
export TMPDIR=/tmp
mkdir -p gpurun_out/ebm_pmc
bash tools/gpu_ebm_check.sh || exit 1
timeout -k 5 60 rocprofv3 -L > gpurun_out/ebm_pmc/counters.txt 2>&1; grep -o "SQ_[A-Z_]*MFMA[A-Z_0-9]*" gpurun_out/ebm_pmc/counters.txt | sort -u | tr '\n' ' '; echo
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ebm_pmc/trace -o run --output-format csv -- python3 tools/ebm_pmc.py > gpurun_out/ebm_pmc/trace.log 2>&1 || exit 1
grep "TFLOP" gpurun_out/ebm_pmc/trace.log
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/ebm_pmc/pmc -o run --output-format csv -- python3 tools/ebm_pmc.py > gpurun_out/ebm_pmc/pmc.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/ebm_pmc/pmc/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r["Kernel_Name"]
    if "prior_chain" in k or "ebm_reg" in k:
        agg[k[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, dict(v))
PY
