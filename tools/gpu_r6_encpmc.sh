# round 6: SQ wave-cycle breakdown (wait / issue-stall / active) of the encoder's first-layer passes, CelebA-HQ B=8, 64
export TMPDIR=/tmp
O=gpurun_out/${1:-r6ep}; mkdir -p $O
for B in 8 64; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $O/pmc_$B -o run --output-format csv -- python3 tools/encoder_profile.py celebaHQ $B 1 > $O/pmc_$B.log 2>&1 || exit 1
done
