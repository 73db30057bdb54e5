# round-3 first box: limb-GEMM stagger A/B (tools/gemm_bench), then the round refresh (tools/gpu_round.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/gemm_bench 128 > gpurun_out/gemm_bench_stag.txt 2>&1 || { cat gpurun_out/gemm_bench_stag.txt; exit 1; }
cat gpurun_out/gemm_bench_stag.txt
bash tools/gpu_round.sh
