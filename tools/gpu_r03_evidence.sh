#!/bin/bash
# Round-3 evidence on one box, each step under its own limit (tools/gpu_steps.sh stops at a
# crash / timeout): smoke, the default bench line, the kernel-trace profile of the bench, the
# PMC traffic + SQ passes of the roofline kernels, then the TPS, ATLAS, training and dopri5 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "smoke|400|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r03_bench|600|python bench.py > gpurun_out/r03_bench.json" \
  "r03_prof|600|bash tools/gpu_prof.sh" \
  "r03_pmc|700|bash tools/roof_pmc.sh" \
  "r03_tps|400|python bench.py --tps --frames 100 --batch 16 > gpurun_out/r03_bench_tps.json" \
  "r03_atlas|500|python bench.py --frames 250 --crop 256 --batch 1 --lanes 1 --sweep-batches '' --no-f32-line --cpu-seconds 20 > gpurun_out/r03_bench_atlas.json" \
  "r03_train|600|python bench.py --train --batch 8 > gpurun_out/r03_bench_train.json" \
  "r03_dopri5|500|python bench.py --sampler dopri5 > gpurun_out/r03_bench_dopri5.json"
