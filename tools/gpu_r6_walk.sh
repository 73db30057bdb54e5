# round 6: the 4 x 4 conv walk for the encoder's convs -- tests, A/B, FETCH per conv
export TMPDIR=/tmp
O=gpurun_out/${1:-r6m}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "encoder or xemb or celebaHQ_q or amortizer or checkpoint or pack_conv or q_update or qtrain" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/enc_ab.py DAMC_ENC_WALK 1,0 celebaHQ:64 celebaHQ:8 celeba64:256 cifar10:128 > $O/walk_ab.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/walk_ab.txt
for wv in 1 0; do
  DAMC_ENC_WALK=$wv timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/f_$wv -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 64 1 > /dev/null 2>&1 || exit 1
  DAMC_ENC_WALK=$wv timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/t_$wv -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 64 2 > /dev/null 2>&1 || exit 1
  f=$(find $O/t_$wv -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_tail.py $f "conv3_mfma_kernel<3, 4, false>" "CelebA-HQ encoder B=64, DAMC_ENC_WALK=$wv: one call" > $O/enc_hq64_walk$wv.txt || exit 1
  grep -E "gemm_x3|span" $O/enc_hq64_walk$wv.txt
done
python3 - <<'PY'
import csv, glob
for n in ("1", "0"):
    f = glob.glob("gpurun_out/r6m/f_%s/**/*counter_collection.csv" % n, recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "gemm_x3_kernel" in r["Kernel_Name"]]
    print("walk", n, ["%.0f" % (2 * float(r["Counter_Value"]) * 1024 / 1e6) for r in rows[-6:]], "MB FETCH (x2) per conv")
PY
