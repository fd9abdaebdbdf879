#!/bin/bash
# Round 4: wgrad split A/B (tile x target block count) on the training line, the world-1 RCCL
# training trace, the dopri5 line and the B = 1 window's kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python bench.py --train --batch 8 --no-cpu-baseline --steps 8 --warmup 3"
bash tools/gpu_steps.sh \
  "wg_w1_256|100|MDG_WGRAD_WIDE=1 MDG_WGRAD_BLOCKS=256 $T > gpurun_out/wg_w1_256.json" \
  "wg_w0_256|100|MDG_WGRAD_WIDE=0 MDG_WGRAD_BLOCKS=256 $T > gpurun_out/wg_w0_256.json" \
  "wg_w0_384|100|MDG_WGRAD_WIDE=0 MDG_WGRAD_BLOCKS=384 $T > gpurun_out/wg_w0_384.json" \
  "wg_w0_512|100|MDG_WGRAD_WIDE=0 MDG_WGRAD_BLOCKS=512 $T > gpurun_out/wg_w0_512.json" \
  "wg_w1_512|100|MDG_WGRAD_WIDE=1 MDG_WGRAD_BLOCKS=512 $T > gpurun_out/wg_w1_512.json" \
  "trainprof_rccl|200|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "dopri5|150|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r04_bench_dopri5.json" \
  "prof_b1|150|PROF_DIR=gpurun_out/prof_b1 BENCH_ARGS='--batch 1 --lanes 1' bash tools/gpu_prof.sh"
