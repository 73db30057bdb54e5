# team sweep: timing (team vs launch chain), then the sweep parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 120 python3 tools/sweep_profile.py 128 || exit 1
DAMC_SWEEP_TEAM=0 timeout -k 5 120 python3 tools/sweep_profile.py 128 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/team_tests.log 2>&1
rc=$?; tail -5 gpurun_out/team_tests.log; exit $rc
