# split-K grid threshold A/B on the bench's config legs (alternating processes; the workspace is sized by the
# same threshold, so each process sets it before the library loads)
export TMPDIR=/tmp
for r in 1 2; do
  for w in 96 128 192; do
    echo -n "wgs<$w: "
    DAMC_X3_KSPLIT_WGS=$w timeout -k 5 200 python3 -c "
import sys, json, torch
sys.path.insert(0, 'diffusion-amortized-mcmc_amd'); sys.path.insert(0, '.')
import bench
from damc import langevin as lv
legs = bench.config_legs(lv, torch.device('cuda:0'), 416.7)
print(json.dumps({k.split(' (')[0]: v['ms_per_step'] for k, v in legs.items()}))
" 2>/dev/null || exit 1
  done
done
