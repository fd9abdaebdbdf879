#!/bin/bash
# Round-3 closing evidence from the final tree, each step under its own limit (tools/gpu_steps.sh
# stops at a crash / timeout): smoke, the GPU suite, the default bench line, its kernel-trace
# profile, the TPS and training lines (with their CPU baselines) and the training step's trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "smoke|400|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|900|bash tools/gpu_suite.sh" \
  "r03_bench|600|python bench.py > gpurun_out/r03_bench.json" \
  "r03_prof|600|bash tools/gpu_prof.sh" \
  "r03_tps|400|python bench.py --tps --frames 100 --batch 16 > gpurun_out/r03_bench_tps.json" \
  "r03_train|600|python bench.py --train --batch 8 > gpurun_out/r03_bench_train.json" \
  "r03_trainprof|400|bash tools/gpu_train_prof.sh"
