export TMPDIR=/tmp
timeout -k 10 1000 python bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err
rc=$?
tail -c 3000 gpurun_out/bench_r02.json
tail -5 gpurun_out/bench_r02.err
exit $rc
