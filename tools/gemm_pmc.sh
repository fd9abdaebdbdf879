#!/bin/bash
# SQ / TA counter passes over the GEMM microbench (tools/gemm_bench.py MODE): where the main
# loop's cycles go (MFMA busy, waits, issue stalls, VMEM / LDS instruction counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
MODE=${1:-b4}
# PMC_RE: the kernel-name filter (default the GEMM kernels); PMC_DIR: the output directory
RE=${PMC_RE:-gemm_}
OUT=${PMC_DIR:-gpurun_out/pmc_gemm}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "$RE" --output-format csv \
    -d $OUT -o p$i -- python tools/gemm_bench.py $MODE > $OUT/log_$i.txt 2>&1 || echo "pass $i rc=$?"
done
echo done
