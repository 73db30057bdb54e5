# A/B of the headline bench line across per-call environment switches of the library, alternated in separate
# processes on one box: bash tools/gpu_ab_env.sh "VAR=val[,VAR=val]" ...  ("default" = no switch)
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in default "$@"; do
    envs=()
    [ "$v" = default ] || IFS=',' read -ra envs <<< "$v"
    echo -n "$v: "
    env "${envs[@]}" timeout -k 5 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernel_classes']; print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], 'proj_fwd', k['proj_fwd']['avg_ms'], 'smallc_fwd', k['smallc_fwd']['avg_ms'], 'smallc_dgrad', k['smallc_dgrad']['avg_ms'])" || exit 1
  done
done
