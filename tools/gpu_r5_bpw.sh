# round 5: split-K sign blocks per workgroup (DAMC_X3_KSPLIT_BPW) at the per-rank batches, interleaved
export TMPDIR=/tmp
O=gpurun_out/${1:-r5bp}; mkdir -p $O
timeout -k 10 300 python tools/post_step_ab.py DAMC_X3_KSPLIT_BPW 1,2,4 16 32 2>/dev/null | tee $O/bpw_ab.txt || exit 1
