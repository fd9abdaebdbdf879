#!/bin/bash
# Round 4: the training step's kernel trace (plain, and with the world-1 RCCL bucket
# all-reduces captured in the graph), the headline bench line and its kernel trace, and kernel
# traces of the small-M windows (B = 1 one chain; TPS B = 16 x T = 100).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "trainprof|200|bash tools/gpu_train_prof.sh" \
  "trainprof_rccl|200|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "bench|240|python bench.py > gpurun_out/r04_bench.json" \
  "prof|200|bash tools/gpu_prof.sh" \
  "prof_b1|150|PROF_DIR=gpurun_out/prof_b1 BENCH_ARGS='--batch 1 --lanes 1' bash tools/gpu_prof.sh" \
  "dopri5|150|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r04_bench_dopri5.json"
