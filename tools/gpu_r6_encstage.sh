# round 6: the first layer's window staging with 8 loads in flight per thread: encoder GPU tests, then one CelebA-HQ
# B=8 / B=64 and CIFAR B=128 call's dispatches
export TMPDIR=/tmp
O=gpurun_out/${1:-r6es}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k 'encoder or Encoder or strong' tests/test_gpu_configs.py tests/test_gpu_amortizer.py tests/test_gpu_strong_scaling.py > $O/tests.log 2>&1 || exit 1
for c in "celebaHQ 8" "celebaHQ 64" "cifar10 128"; do
  set -- $c
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc_$1_$2 -o run --output-format csv -- python3 tools/encoder_profile.py $1 $2 3 > $O/enc_$1_$2.log 2>&1 || exit 1
  f=$(find $O/enc_$1_$2 -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_tail.py $f "conv3_mfma_kernel<3, 4, true>|conv3_in_fused|conv3_stats" "$1 encoder B=$2: one call" > $O/enc_$1_$2_dispatches.txt || exit 1
done
