# round 6: km_skinny_kernel at 33-64 rows, DAMC_KM_SKINNY_MT=2 (one 64-row workgroup of <2>) vs the default (two 32-row workgroups of <1>): kernel stats
export TMPDIR=/tmp
O=gpurun_out/${1:-r6km}; mkdir -p $O
for v in 2 1; do
  DAMC_KM_SKINNY_MT=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/mt$v -o run --output-format csv -- python3 tools/cfg_profile.py _netG_svhn 100 64 32 64 20 > $O/mt$v.log 2>&1 || exit 1
done
