# P16 limb-GEMM A/B + the sweep end-point distances (printed by the amortizer tests)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 ./tools/gemm_bench 128 > gpurun_out/gemm_p16.txt 2>&1; rc=$?; cut -c1-330 gpurun_out/gemm_p16.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_amortizer.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/amortizer_s.log 2>&1
rc=$?; grep "sweep end" gpurun_out/amortizer_s.log; tail -2 gpurun_out/amortizer_s.log; exit $rc
