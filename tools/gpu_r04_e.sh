#!/bin/bash
# Round 4: the fused spatial kernel standalone (MFMA vs VALU epilogue, each at both launch-bound
# settings via a diagnostic library), the training step's kernel trace, the headline bench line
# and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "spa_mf4|60|MDG_SPA_MFMA=1 python tools/gemm_bench.py spa" \
  "spa_valu3|60|MDG_SPA_MFMA=0 python tools/gemm_bench.py spa" \
  "spa_mf3|60|MDG_LIB_PATH=diaglib/spa_lb.so MDG_SPA_MFMA=1 python tools/gemm_bench.py spa" \
  "spa_valu4|60|MDG_LIB_PATH=diaglib/spa_lb.so MDG_SPA_MFMA=0 python tools/gemm_bench.py spa" \
  "trainprof|200|bash tools/gpu_train_prof.sh" \
  "bench|240|python bench.py > gpurun_out/r04_bench.json" \
  "prof|200|bash tools/gpu_prof.sh"
