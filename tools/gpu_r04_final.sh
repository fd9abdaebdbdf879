#!/bin/bash
# Round-4 closing evidence from the final tree, each step under its own limit (tools/gpu_steps.sh
# stops at a crash / timeout): smoke, the GPU suite (parity errors logged), the default bench line
# and its kernel-trace profile, the training line (CPU baseline) and its step trace, the world-1
# RCCL bucket rehearsal trace, the dopri5 line and the B = 1 window trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "smoke|400|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|960|bash tools/gpu_suite.sh" \
  "r04_bench|400|python bench.py > gpurun_out/r04_bench.json" \
  "r04_prof|300|bash tools/gpu_prof.sh" \
  "r04_train|400|python bench.py --train --batch 8 > gpurun_out/r04_bench_train.json" \
  "r04_trainprof|300|bash tools/gpu_train_prof.sh" \
  "r04_trainprof_rccl|300|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "r04_dopri5|300|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r04_bench_dopri5.json" \
  "r04_prof_b1|300|PROF_DIR=gpurun_out/prof_b1 BENCH_ARGS='--batch 1 --lanes 1' bash tools/gpu_prof.sh"
