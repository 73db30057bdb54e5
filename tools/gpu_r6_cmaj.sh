# round 6: the channel-major K walk (V 269) against the tap-major default (261) on the encoder's limb-gathering path
# (DAMC_ENC_F32A=0), CelebA-HQ: is the encoder conv bound by L2 misses of the stride-2 gather?
export TMPDIR=/tmp
O=gpurun_out/${1:-r6l}; mkdir -p $O
export DAMC_ENC_F32A=0 DAMC_ENC_HEAD=0
for r in 1 2; do
  for t in . abtree/v269; do
    timeout -k 10 120 python tools/enc_tree.py $t celebaHQ:64 celebaHQ:8 >> $O/cmaj_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/cmaj_ab.txt
for t in . abtree/v269; do
  n=$(basename $t)
  timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/tr_$n -o run --output-format csv -- python3 tools/enc_tree.py $t celebaHQ:64 > /dev/null 2>&1 || exit 1
  f=$(find $O/tr_$n -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_tail.py $f "conv3_mfma_kernel<3, 4, false>|conv3_apply" "tree $n HQ B=64" | grep -E "gemm_x3|span|conv3" 
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/f_$n -o run --output-format csv -- python3 tools/enc_tree.py $t celebaHQ:64 > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob
for n in (".", "v269"):
    f = glob.glob("gpurun_out/r6l/f_%s/**/*counter_collection.csv" % n, recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "gemm_x3_kernel" in r["Kernel_Name"]]
    print(n, ["%.0f" % (2 * float(r["Counter_Value"]) * 1024 / 1e6) for r in rows[-6:]], "MB (x2 corrected)")
PY
