# chain-kernel segment stamps (DAMC_CHAIN_TRACE) for DAMC_CHAIN_DBG variants (1024 = wait for the first chunk's loads)
mkdir -p gpurun_out
for d in "$@"; do
  echo "== dbg=$d"
  DAMC_CHAIN_DBG=$d DAMC_CHAIN_TRACE=gpurun_out/chain_trace.bin timeout -k 5 120 python3 tools/sweep_profile.py 128 > gpurun_out/ctrace.log 2>&1 || exit 1
  python3 tools/chain_stamps.py gpurun_out/chain_trace.bin | tail -8
done
