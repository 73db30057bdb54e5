# team sweep: timing (team vs launch chain), then the sweep parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 120 python3 tools/sweep_profile.py 128 || exit 1
DAMC_SWEEP_TEAM=0 timeout -k 5 120 python3 tools/sweep_profile.py 128 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_ops.py tests/test_gpu_configs.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/team_tests.log 2>&1
rc=$?; grep -E "team vs chain|passed|failed|Error" gpurun_out/team_tests.log | tail -12; exit $rc
