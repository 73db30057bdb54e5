export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_gpu_strong_scaling.py "tests/test_gpu_optim.py::test_adam_step_counters_with_partial_gradients" "tests/test_gpu_amortizer.py::test_classifier_free_guidance_matches_stock_modules" -s > gpurun_out/r6a/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6a/tests.log; exit $rc
