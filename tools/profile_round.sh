#!/bin/bash
# Refresh the committed profiles on an MI355X box (run through gpurun from the repo root):
#   rocprofv3 kernel-trace stats of a short bench run, then FETCH_SIZE and WRITE_SIZE in separate
#   --pmc passes (MI355X_MICROARCH.md §HBM), reduced per kernel class by tools/pmc_traffic.py.
set -e
OUT=${1:-gpurun_out/prof}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/bench_under_rocprof.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" > "$OUT/pmc_traffic.txt"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE -d "$OUT/clock" -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extras > "$OUT/clock.log" 2>&1
(cd tools && python3 pmc_clock.py "../$OUT/clock" "../$OUT/trace") > "$OUT/clock.txt"
