#!/bin/bash
# HBM-traffic counter passes for the bench roofline kernels: FETCH_SIZE and WRITE_SIZE in
# separate runs (they do not fit one TCC pass), counters only (no tracing).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# ROOF_ARGS="B T L" selects another shape (e.g. "1 250 256", ATLAS), written to pmc_roof_B_T_L
D=gpurun_out/pmc_roof${ROOF_ARGS:+_${ROOF_ARGS// /_}}
mkdir -p $D
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "gemm_bf16_b4|attn_temporal_bf16|gemm_rowln|mlp_rowln|mlp_ws2|rowln_qkv" \
    --output-format csv -d $D -o $C -- python tools/roof_kernels.py ${ROOF_ARGS:-} \
    > $D/log_$C.txt 2>&1 || exit $?
done
# SQ pass: where the roofline kernels' cycles go (VALU vs MFMA instructions, MFMA-busy, waits)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "gemm_bf16_b4|attn_temporal_bf16|gemm_rowln|mlp_rowln|mlp_ws2|rowln_qkv|gemm_qkv_attn_spatial" \
  --output-format csv -d $D -o SQ -- python tools/roof_kernels.py ${ROOF_ARGS:-} > $D/log_SQ.txt 2>&1 || exit $?
echo done
