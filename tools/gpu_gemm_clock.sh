# effective clock of each limb-GEMM variant in tools/gemm_bench (GRBM_GUI_ACTIVE pass + kernel-trace pass)
export TMPDIR=/tmp
mkdir -p gpurun_out/gclk
timeout -s KILL 120 rocprofv3 --kernel-trace -d gpurun_out/gclk/trace -o run --output-format csv -- ./tools/gemm_bench 128 > gpurun_out/gclk/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d gpurun_out/gclk/clock -o run --output-format csv -- ./tools/gemm_bench 128 > gpurun_out/gclk/clock.log 2>&1 || exit 1
grep -A6 "best-of" gpurun_out/gclk/trace.log | cut -c1-200
python3 tools/pmc_clock_kernels.py gpurun_out/gclk/clock gpurun_out/gclk/trace gemm_x3
