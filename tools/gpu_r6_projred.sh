# round 6: the fused split-K reduce + output projection with its row divisions hoisted: bitwise tests, then one
# posterior step's dispatches at CIFAR B=16 and SVHN B=64
export TMPDIR=/tmp
O=gpurun_out/${1:-r6pr}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "projection or ksplit or split_k" tests/test_gpu_langevin.py > $O/tests.log 2>&1 || exit 1
for cfg in "_netG_cifar10 128 128 32 16 cifar10_b16" "_netG_svhn 100 64 32 64 svhn_b64"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/$6 -o run --output-format csv -- python3 tools/cfg_profile.py $1 $2 $3 $4 $5 4 > $O/$6.log 2>&1 || exit 1
  f=$(find $O/$6 -name '*kernel_trace.csv' | head -1)
  python3 tools/dispatch_list.py $f "$6: one posterior step" > $O/$6_dispatches.txt || exit 1
done
