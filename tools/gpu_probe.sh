# limb-GEMM timing probes (tools/gemm_bench: no DMA / first-tile reads only / MFMA only) + the new G-update test
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/gemm_bench 128 > gpurun_out/gemm_probe.txt 2>&1 || { cat gpurun_out/gemm_probe.txt; exit 1; }
cat gpurun_out/gemm_probe.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -k "second_backward" -x -v --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; tail -3 gpurun_out/t2.log; exit $rc
