export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
timeout -k 10 900 python -u -m pytest tests/test_gpu_amortizer.py tests/test_gpu_configs.py tests/test_gpu_training.py tests/test_gpu_checkpoint.py tests/test_gpu_dropin.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r3d/tests.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r3d/tests.log | tail -2; grep -E "^FAILED|Error" gpurun_out/r3d/tests.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-torch-g > gpurun_out/r3d/bench.json 2> gpurun_out/r3d/bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r3d/bench.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['amortizer']))"
