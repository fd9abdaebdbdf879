#!/bin/bash
# SQ counter pass over the temporal attention kernel at the bench shape (counters only), for the
# tree's library and, when given, a second one (MDG_LIB_PATH): MFMA-busy, VALU and wait shares.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/pmc
for L in new ${OLD_LIB:+old}; do
  if [ $L = old ]; then export MDG_LIB_PATH=$OLD_LIB; else unset MDG_LIB_PATH; fi
  timeout -k 10 120 python tools/attn_bench.py 20 | tail -1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/pmc -o attn_$L -- python tools/attn_bench.py 5 > gpurun_out/pmc/attn_log_$L.txt 2>&1 \
    || { echo "pmc rc=$?"; exit 1; }
done
echo done
