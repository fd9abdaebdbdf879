#!/bin/bash
# SQ counter pass over the temporal attention kernel at the bench shape (counters only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d gpurun_out/pmc -o attn -- python tools/attn_bench.py 5 > gpurun_out/pmc/attn_log.txt 2>&1
