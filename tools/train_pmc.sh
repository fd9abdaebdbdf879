#!/bin/bash
# PMC passes over the config-3 training step (bench.py --train): HBM traffic (FETCH_SIZE,
# WRITE_SIZE in separate runs) and SQ issue counters for the block stack's GEMM, weight-gradient
# and attention-backward kernels.  Counters only, one pass per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
D=${PMC_DIR:-gpurun_out/pmc_train}
mkdir -p $D
RX=${PMC_REGEX:-"gemm_bf16_b4|wgrad_bf16|split_sum|attn_bwd_fused|attn_temporal_bf16|mlp_rowln|mlp_ws2|gemm_rowln"}
ARGS="bench.py --train --batch 8 --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d $D -o $C -- \
    python $ARGS > $D/log_$C.txt 2>&1 || exit $?
done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "$RX" --output-format csv -d $D -o SQ -- python $ARGS > $D/log_SQ.txt 2>&1 || exit $?
echo done
