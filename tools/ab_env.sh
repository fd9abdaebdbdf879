#!/bin/bash
# Same-box A/B of the training step under two environment settings: AB_ENV_A / AB_ENV_B (e.g.
# "MDG_TRAIN_WGRAD_STREAM=0"), alternating twice; prints ms per step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for V in A B; do
    eval "E=\${AB_ENV_$V:-}"
    timeout -k 10 300 env $E python -u bench.py --train --batch 8 --steps ${AB_STEPS:-10} --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_env_$V.json 2> gpurun_out/ab_env_$V.err || { tail -5 gpurun_out/ab_env_$V.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_env_$V.json').read().strip().splitlines()[-1]);print('$V [$E]', d['ms_per_step'], d['value'])"
  done
done
