# round 5: the skinny-kernel bitwise tests, then the per-rank legs (cfg_versions) with km_skinny for M <= 64 vs the tiled
# kernel (DAMC_KM_SKINNY=0), interleaved, and a dispatch trace of SVHN B=64 and CIFAR B=16
export TMPDIR=/tmp
O=gpurun_out/${1:-r5l}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_langevin.py -k "skinny or sharded or split" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "" "DAMC_KM_SKINNY=0"; do
    echo "[$v]" >> $O/legs_ab.txt
    env $v timeout -k 5 120 python3 tools/cfg_versions.py . svhn64 celeba32 cifar16 >> $O/legs_ab.txt 2>&1 || exit 1
  done
done
cat $O/legs_ab.txt | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/svhn -o run --output-format csv -- python3 tools/cfg_profile.py _netG_svhn 100 64 32 64 > $O/svhn.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/b16 -o run --output-format csv -- python3 tools/b16_profile.py 16 > $O/b16.log 2>&1 || exit 1
