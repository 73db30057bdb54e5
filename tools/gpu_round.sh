# round refresh on one MI355X: every GPU test, the default bench line, then tools/profile_round.sh's passes
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
tail -c 600 gpurun_out/bench.json
bash tools/profile_round.sh gpurun_out/prof || exit 1
cat gpurun_out/prof/pmc_traffic.txt gpurun_out/prof/clock.txt
# the reverse sweep (Q(x) at B=128, 100 steps) under rocprofv3: the team kernel's share of a sweep
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/sweep -o run --output-format csv -- \
  python3 tools/sweep_profile.py 128 > gpurun_out/prof/sweep_profile.log 2>&1 || exit 1
tail -4 gpurun_out/prof/sweep_profile.log
