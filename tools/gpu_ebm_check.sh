# EBM: prior-chain parity (both engines) and the engine timing sweep over batch sizes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_langevin.py -x -q -k "prior" --timeout 120 --timeout-method thread > gpurun_out/ebm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ebm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/ebm_profile.py
