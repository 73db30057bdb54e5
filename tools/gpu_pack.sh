# conv weight limb packing: the bit-exact test, encoder / Q tests, then the amortizer leg of the bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "pack or encoder or q_" > gpurun_out/pack_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" gpurun_out/pack_tests.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/pack_bench.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/pack_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['amortizer'])"
