# round 6: the KREG store without the s_nop -- bitwise gates, then the per-rank step against round 5's numbers
export TMPDIR=/tmp
O=gpurun_out/${1:-r6g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_langevin.py::test_f32a_posterior_is_bitwise" \
  "tests/test_gpu_langevin.py::test_split_k_is_bitwise_the_unsplit_kernel" \
  "tests/test_gpu_langevin.py::test_fused_output_projection_is_bitwise" \
  tests/test_gpu_strong_scaling.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/post_step_ab.py DAMC_NOP_AB 0 16 svhn:64 > $O/step.txt 2>&1 || exit 1
cat $O/step.txt
