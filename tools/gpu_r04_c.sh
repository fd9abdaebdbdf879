#!/bin/bash
# Round 4: the training step's kernel trace (plain, and with the world-1 RCCL bucket
# all-reduces captured in the graph), the headline bench line and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "trainprof|240|bash tools/gpu_train_prof.sh" \
  "trainprof_rccl|240|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "bench|300|python bench.py > gpurun_out/r04_bench.json" \
  "prof|240|bash tools/gpu_prof.sh"
