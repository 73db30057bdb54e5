# A/B of the sweep: default library vs the alternative build(s) given as arguments (DAMC_LIB_PATH), interleaved
for r in 1 2; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset DAMC_LIB_PATH; else export DAMC_LIB_PATH=$lib; fi
    echo -n "$lib: "; timeout -k 5 120 python3 tools/sweep_profile.py 128 2>&1 | grep -o "'us_per_denoise_step': [0-9.]*\|denoise_chain.*\|sweep_hyper.*" | tr '\n' ' ' || exit 1; echo
  done
done
