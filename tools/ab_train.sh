#!/bin/bash
# Same-box A/B of the training step: the tree's library vs ablib/old.so (tools/build_ab.sh),
# alternating twice; optional microbench AB_MICRO (a python script) run under both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export MDG_LIB_PATH=$PWD/ablib/old.so; else unset MDG_LIB_PATH; fi
    if [ -n "${AB_MICRO:-}" ]; then
      echo "== micro $L"; timeout -k 10 120 python $AB_MICRO 2>&1 | tail -${AB_MICRO_LINES:-8} || exit $?
    fi
    timeout -k 10 300 python -u bench.py --train --batch 8 --steps ${AB_STEPS:-10} --warmup 2 --no-cpu-baseline \
      > gpurun_out/ab_train_$L.json 2> gpurun_out/ab_train_$L.err || { tail -5 gpurun_out/ab_train_$L.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_train_$L.json').read().strip().splitlines()[-1]);print('$L', d['ms_per_step'], d['value'])"
  done
done
