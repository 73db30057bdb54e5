# per-block chain kernel times of the Q(x) sweep under rocprofv3, for DAMC_CHAIN_DBG variants given as arguments
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in "$@"; do
  DAMC_CHAIN_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ct$d -o run --output-format csv -- python3 tools/sweep_profile.py 128 > gpurun_out/ct$d.log 2>&1 || exit 1
  echo "dbg=$d"; grep -o "'us_per_denoise_step': [0-9.]*" gpurun_out/ct$d.log; python3 tools/chain_trace.py $(find gpurun_out/ct$d -name "*kernel_trace.csv" | head -1)
done
