#!/bin/bash
# Round-5 closing evidence from the final tree, in three gpurun calls (each step under its own
# limit; tools/gpu_steps.sh stops at a crash / timeout):
#   a: smoke, the GPU suite (parity errors logged);
#   b: the default bench line, its kernel-trace profile, the bench roofline kernels' PMC passes,
#      the B = 1 window line and trace, the TPS B = 16 line;
#   c: the training line (CPU baseline), its step trace and PMC / SQ passes, the world-1 RCCL
#      bucket rehearsal trace, the dopri5 line.
# Summaries: tools/make_profiles.py 05, tools/train_profile_md.py 05, tools/rccl_overlap_trace.py,
# tools/pmc_summary.py.   usage: tools/gpu_r05_final.sh a|b|c
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
case "${1:-}" in
a) bash tools/gpu_steps.sh \
  "smoke|400|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|960|bash tools/gpu_suite.sh" ;;
b) bash tools/gpu_steps.sh \
  "r05_bench|400|python bench.py > gpurun_out/r05_bench.json" \
  "r05_prof|300|bash tools/gpu_prof.sh" \
  "r05_roofpmc|300|bash tools/roof_pmc.sh" \
  "r05_b1|200|python bench.py --batch 1 --lanes 1 --steps 3 --warmup 1 --sweep-batches '' --no-f32-line > gpurun_out/r05_bench_b1.json" \
  "r05_prof_b1|200|PROF_DIR=gpurun_out/prof_b1 BENCH_ARGS='--batch 1 --lanes 1' bash tools/gpu_prof.sh" \
  "r05_tps|200|python bench.py --tps --frames 100 --batch 16 --steps 3 --warmup 1 --sweep-batches '' --no-f32-line > gpurun_out/r05_bench_tps.json" ;;
c) bash tools/gpu_steps.sh \
  "r05_train|300|python bench.py --train --batch 8 > gpurun_out/r05_bench_train.json" \
  "r05_trainprof|300|bash tools/gpu_train_prof.sh" \
  "r05_trainpmc|400|bash tools/train_pmc.sh" \
  "r05_trainprof_rccl|300|PROF_DIR=gpurun_out/prof_train_rccl BENCH_ARGS=--train-rccl1 bash tools/gpu_train_prof.sh" \
  "r05_dopri5|200|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r05_bench_dopri5.json" ;;
*) echo "usage: $0 a|b|c"; exit 2 ;;
esac
