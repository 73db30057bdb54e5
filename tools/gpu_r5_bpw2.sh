# round 5: DAMC_X3_KSPLIT_BPW pinned to 2 against the default rule on the per-rank legs (cfg_versions), interleaved
export TMPDIR=/tmp
O=gpurun_out/${1:-r5b2}; mkdir -p $O
for r in 1 2; do
  for v in "" "DAMC_X3_KSPLIT_BPW=2"; do
    echo "[$v]" >> $O/bpw2_ab.txt
    env $v timeout -k 5 120 python3 tools/cfg_versions.py . celeba32 svhn64 cifar16 >> $O/bpw2_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/bpw2_ab.txt
