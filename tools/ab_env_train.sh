#!/bin/bash
# Same-box A/B of the training step on one library, an env knob off / on, alternating twice:
#   AB_VAR=MDG_SPATIAL_BWD_QUADH bash tools/ab_env_train.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    env "$AB_VAR=$v" timeout -k 10 300 python -u bench.py --train --batch 8 --steps ${AB_STEPS:-10} --warmup 2 \
      --no-cpu-baseline > gpurun_out/ab_env_train_$v.json 2> gpurun_out/ab_env_train_$v.err \
      || { tail -5 gpurun_out/ab_env_train_$v.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_env_train_$v.json').read().strip().splitlines()[-1]);print('$AB_VAR=$v', d['ms_per_step'], d['value'])"
  done
done
