# A/B of the headline bench line: default library vs the alternative build(s) given as arguments
# (DAMC_LIB_PATH), alternated in separate processes on one box
export TMPDIR=/tmp
for r in 1 2 3; do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then unset DAMC_LIB_PATH; else export DAMC_LIB_PATH=$lib; fi
    echo -n "$lib: "
    timeout -k 5 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" || exit 1
  done
done
