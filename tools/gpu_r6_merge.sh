# round 6: tree InstanceNorm merge; encoder GPU tests, then host/GPU time per encoder call and HQ B=8 dispatches
export TMPDIR=/tmp
O=gpurun_out/${1:-r6u}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_amortizer.py tests/test_gpu_training.py tests/test_gpu_strong_scaling.py -k "encoder or Q or q_ or xemb or amortizer or strong" > $O/tests.txt 2>&1; tail -3 $O/tests.txt
for cfg in "cifar10 128" "celebaHQ 8" "celebaHQ 64"; do
  set -- $cfg
  timeout -k 10 120 python tools/enc_hosttime.py $1 $2 30 > $O/host_$1_$2.txt 2>&1 || exit 1
  grep "back-to-back" $O/host_$1_$2.txt
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc_hq8 -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ 8 3 > $O/enc_hq8.log 2>&1 || exit 1
f=$(find $O/enc_hq8 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_tail.py $f "conv3_mfma_kernel<3, 4, true>" "celebaHQ encoder B=8: one call" > $O/enc_hq8_dispatches.txt || exit 1
cat $O/enc_hq8_dispatches.txt
