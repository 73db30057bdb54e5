# round 6: the split-K in-GEMM fix-up -- bitwise gates, then the per-rank step A/B against the reduce launches
export TMPDIR=/tmp
O=gpurun_out/${1:-r6b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_langevin.py::test_split_k_is_bitwise_the_unsplit_kernel" \
  "tests/test_gpu_langevin.py::test_f32a_posterior_is_bitwise" \
  "tests/test_gpu_langevin.py::test_fused_output_projection_is_bitwise" \
  "tests/test_gpu_langevin.py::test_sharded_chains_are_bitwise_identical" \
  tests/test_gpu_strong_scaling.py tests/test_gpu_graph.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/post_step_ab.py DAMC_X3_FIXUP 1,0 16 128 svhn:64 celeba64:32 celebaHQ:8 > $O/fixup_ab.txt 2>&1 || exit 1
cat $O/fixup_ab.txt
