#!/bin/bash
# Same-box timing of several environment variants of the inference bench line, alternating
# AB_REPS (1) rounds: AB_VARIANTS is a ';'-separated list of environment settings ("-" = none).
#   AB_VARIANTS="-;MDG_MLP_WS=2;MDG_MLP_WS=2 MDG_LIB_PATH=$PWD/ablib/diag2.so" bash tools/ab_multi.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "$AB_VARIANTS"
for rep in $(seq ${AB_REPS:-1}); do
  i=0
  for E in "${VS[@]}"; do
    [ "$E" = "-" ] && E=""
    eval "env $E timeout -k 10 300 python -u bench.py --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline --no-f32-line \
      --sweep-batches '' ${AB_ARGS:-}" > gpurun_out/abm_$i.json 2> gpurun_out/abm_$i.err || { tail -5 gpurun_out/abm_$i.err; exit 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/abm_$i.json') if l.startswith('{')][-1]);print('[$E]', d['value'], d['us_per_denoise_step'], [r['avg_launch_us'] for r in [d['roofline']]+(d['roofline_more'] or [])])"
    i=$((i+1))
  done
done
