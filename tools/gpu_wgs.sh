# split-K workgroup threshold A/B (DAMC_X3_KSPLIT_WGS): per-rank posterior step timings at small batch
export TMPDIR=/tmp
for w in 128 256 512 128 256; do
  export DAMC_X3_KSPLIT_WGS=$w
  echo "== ksplit below $w workgroups"
  for B in 8 16 32 64; do timeout -k 10 120 python3 tools/b16_profile.py $B 2>&1 | grep "per posterior" || exit 1; done
done
