# round 6: the sweep's hyper GEMM with parts switched off (DAMC_SWEEP_HYPER_DBG, timing only), then the gate's
# sigmoid on exp2 / rcp against expf + IEEE division (DAMC_SWEEP_HYPER_SIGMOID=exact): tests, A/B, rocprof
export TMPDIR=/tmp
O=gpurun_out/${1:-r6hd}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_amortizer.py tests/test_gpu_configs.py -k "sweep or hyper or team or amortizer or Q" > $O/tests.txt 2>&1; tail -1 $O/tests.txt
timeout -k 10 180 python tools/sweep_ab.py 128 DAMC_SWEEP_HYPER_SIGMOID=fast DAMC_SWEEP_HYPER_SIGMOID=exact > $O/sig_ab.txt 2>&1 || exit 1
grep sweep $O/sig_ab.txt
for v in fast exact; do
  DAMC_SWEEP_HYPER_SIGMOID=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/p_$v -o run --output-format csv -- python3 tools/sweep_profile.py 128 > $O/p_$v.log 2>&1 || exit 1
  python3 tools/kstats.py $(find $O/p_$v -name '*kernel_stats.csv' | head -1) 12 | grep -E "hyper|ctx" | sed "s/^/$v: /"
done
