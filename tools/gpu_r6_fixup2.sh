# round 6: fix-up timeline + A/B (no tests: quick iteration), then the bitwise gate
export TMPDIR=/tmp
O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 120 python tools/fixup_timeline.py 16 > $O/timeline.txt 2>&1 || exit 1
cat $O/timeline.txt
timeout -k 10 300 python -u tools/post_step_ab.py DAMC_X3_FIXUP 1,0 16 svhn:64 celeba64:32 celebaHQ:8 > $O/fixup_ab.txt 2>&1 || exit 1
cat $O/fixup_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_langevin.py::test_split_k_is_bitwise_the_unsplit_kernel" tests/test_gpu_strong_scaling.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
