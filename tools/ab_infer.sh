#!/bin/bash
# Same-box A/B of the inference bench line: each argument is "name|env|bench args"; every variant
# runs twice, alternating.  Prints frames/s and ms per window.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; args=${rest#*|}
    timeout -k 10 300 env $envs python -u bench.py --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline --no-f32-line \
      --sweep-batches "" $args > gpurun_out/abi_$name.json 2> gpurun_out/abi_$name.err || { tail -5 gpurun_out/abi_$name.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abi_$name.json').read().strip().splitlines()[-1]);print('$name', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
