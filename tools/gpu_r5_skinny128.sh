# round 5: skinny first-layer kernels up to 128 rows: bitwise tests, then the headline step and B=16 A/B (same box)
export TMPDIR=/tmp
O=gpurun_out/${1:-r5s}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_langevin.py -k "skinny or sharded or split" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "" "DAMC_X3_SKINNY_ROWS=32 DAMC_KM_SKINNY_ROWS=64"; do
    echo "[$v]" >> $O/ab.txt
    env $v timeout -k 5 120 python3 tools/cfg_versions.py . cifar128 cifar16 >> $O/ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/ab.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/cfg_versions.py . cifar128 > /dev/null 2>&1 || exit 1
