# split-K register slab layout vs row-major: the per-rank posterior step timings only
export TMPDIR=/tmp
for b in 0 1 0 1; do
  if [ $b = 0 ]; then export DAMC_X3_KSLAB_REG=0; else unset DAMC_X3_KSLAB_REG; fi
  echo "== register slab layout: $b"
  for B in 8 16 32; do timeout -k 10 120 python3 tools/b16_profile.py $B 2>&1 | grep "per posterior" || exit 1; done
done
