#!/bin/bash
# Round-5 GPU steps, by name (tools/gpu_steps.sh runs each under its own limit and stops at a
# crash / timeout).  usage: tools/gpu_r05.sh step [step ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
declare -A S=(
  [smoke]="smoke|400|python -c 'import __graft_entry__ as g; g.smoke()'"
  [suite]="suite|960|bash tools/gpu_suite.sh"
  [bench]="bench|400|python bench.py > gpurun_out/bench.json"
  [prof]="prof|300|bash tools/gpu_prof.sh"
  [train]="train|400|python bench.py --train --batch 8 --no-cpu-baseline > gpurun_out/bench_train.json"
  [trainprof]="trainprof|300|bash tools/gpu_train_prof.sh"
  [trainpmc]="trainpmc|900|bash tools/train_pmc.sh"
  [roofpmc]="roofpmc|900|bash tools/roof_pmc.sh"
  [b1]="b1|300|python bench.py --batch 1 --lanes 1 --no-cpu-baseline --sweep-batches '' --no-f32-line > gpurun_out/bench_b1.json"
)
args=()
for n in "$@"; do
  if [ -n "${S[$n]:-}" ]; then args+=("${S[$n]}"); else args+=("$n"); fi
done
bash tools/gpu_steps.sh "${args[@]}"
