export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_langevin.py tests/test_gpu_ops.py tests/test_gpu_checkpoint.py -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_ebm.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_ebm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ebm_profile.py > gpurun_out/ebm_profile.txt 2>&1; cat gpurun_out/ebm_profile.txt
bash tools/chain_dbg.sh > gpurun_out/chain_dbg.txt 2>&1; cat gpurun_out/chain_dbg.txt
