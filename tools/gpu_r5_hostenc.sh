# round 5: encoder tests, the encoder's host time per call, the CelebA-HQ encoder profile, then the bench line
export TMPDIR=/tmp
O=gpurun_out/${1:-r5he}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_amortizer.py tests/test_gpu_checkpoint.py \
  -m gpu -x -v --timeout 120 --timeout-method thread -k "encoder or checkpoint" > $O/enc_tests.log 2>&1
rc=$?; tail -3 $O/enc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/enc_hosttime.py cifar10 128 50 2>/dev/null | tee $O/enc_hosttime.txt || exit 1
bash tools/gpu_r5_hqenc.sh ${1:-r5he} || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -c 300 $O/bench.json
