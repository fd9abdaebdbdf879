#!/bin/bash
# SQ counter pass over one GEMM shape for both tile variants (counters only, no tracing).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc
SHAPE="${SHAPE:-32000 1536 384 0 0}"
for T in 128 256; do
  MDG_GEMM_TILE=$T timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES \
    --output-format csv -d gpurun_out/pmc -o sq_$T -- python tools/gemm_one.py $SHAPE > gpurun_out/pmc/log_$T.txt 2>&1 || exit $?
done
echo done
