# limb-GEMM stagger A/B + the stage-wise encoder-training test
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/gemm_bench 128 > gpurun_out/gemm_bench_stag.txt 2>&1 || { cat gpurun_out/gemm_bench_stag.txt; exit 1; }
cat gpurun_out/gemm_bench_stag.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -k "stagewise" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/stagewise.log 2>&1
rc=$?; grep -i "kink\|IN dy\|passed\|failed" gpurun_out/stagewise.log | tail -30; exit $rc
