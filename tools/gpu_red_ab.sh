# split-K slab A/B (DAMC_X3_KSLAB_OPT bits: 4 the thread-per-32-outputs reduce instead of wave-per-tile)
export TMPDIR=/tmp
for o in 4 0 4 0; do
  export DAMC_X3_KSLAB_OPT=$o
  echo "== opt $o"
  for B in 8 16 32; do timeout -k 10 120 python3 tools/b16_profile.py $B 2>&1 | grep "per posterior" || exit 1; done
  timeout -k 10 200 python3 tools/cfg_profile.py _netG_celebaHQ 128 128 256 8 3 2>&1 | grep "per posterior" || exit 1
done
