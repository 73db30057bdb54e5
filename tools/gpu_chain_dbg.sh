# us per denoise step of the Q(x) sweep (no profiler) for DAMC_CHAIN_DBG variants given as arguments
for d in "$@"; do
  echo -n "dbg=$d "; DAMC_CHAIN_DBG=$d timeout -k 5 120 python3 tools/sweep_profile.py 128 2>&1 | grep -o "'us_per_denoise_step': [0-9.]*" | head -1 || exit 1
done
