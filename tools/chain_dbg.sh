# timing experiment: the reverse sweep's chain kernel with parts switched off (DAMC_CHAIN_DBG, wrong results)
export TMPDIR=/tmp
for d in 0 1 2 3 4 7 8 16 31; do
  echo -n "dbg=$d "
  DAMC_CHAIN_DBG=$d timeout -k 10 120 python tools/sweep_profile.py 128 2>/dev/null | grep -o "'us_per_denoise_step': [0-9.]*"
done
