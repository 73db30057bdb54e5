# round 6 final evidence on HEAD: every GPU test, the default bench line, rocprof stats + PMC traffic + clock of the
# bench (tools/profile_round.sh), one-step dispatch traces at the per-rank batches, a clean default sweep profile, one
# encoder call's dispatches at CelebA-HQ B=8 / B=64 and CIFAR B=128
export TMPDIR=/tmp
O=gpurun_out/${1:-r6z}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 600 $O/bench.json
bash tools/profile_round.sh $O/prof || exit 1
for cfg in "_netG_cifar10 128 128 32 16 cifar10_b16" "_netG_svhn 100 64 32 64 svhn_b64"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/$6 -o run --output-format csv -- python3 tools/cfg_profile.py $1 $2 $3 $4 $5 4 > $O/$6.log 2>&1 || exit 1
  f=$(find $O/$6 -name '*kernel_trace.csv' | head -1)
  python3 tools/dispatch_list.py $f "$6: one posterior step (round 6 end, HEAD)" > $O/$6_dispatches.txt || exit 1
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/sweep -o run --output-format csv -- python3 tools/sweep_profile.py 128 > $O/sweep.log 2>&1 || exit 1
for c in "celebaHQ 8" "celebaHQ 64" "cifar10 128"; do
  set -- $c
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc_$1_$2 -o run --output-format csv -- python3 tools/encoder_profile.py $1 $2 3 > $O/enc_$1_$2.log 2>&1 || exit 1
  f=$(find $O/enc_$1_$2 -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_tail.py $f "conv3_mfma_kernel<3, 4, true>|conv3_in_fused|conv3_stats" "$1 encoder B=$2: one call" > $O/enc_$1_$2_dispatches.txt || exit 1
done
echo done
