# split-K limb GEMM: generator / training parity tests, then the bench's config legs (split at small batch) vs
# DAMC_X3_KSPLIT=0 (unsplit) in alternating processes
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_langevin.py tests/test_gpu_training.py tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_checkpoint.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ksplit_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ksplit_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for ks in 1 0; do
    echo -n "ksplit=$ks: "
    DAMC_X3_KSPLIT=$ks timeout -k 5 200 python3 -c "
import sys, json, torch
sys.path.insert(0, 'diffusion-amortized-mcmc_amd'); sys.path.insert(0, '.')
import bench
from damc import langevin as lv
legs = bench.config_legs(lv, torch.device('cuda:0'), 416.7)
print(json.dumps({k: (v['ms_per_step'], v['frac_of_peak']) for k, v in legs.items()}))
" 2>/dev/null || exit 1
  done
done
