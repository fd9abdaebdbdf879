#!/bin/bash
# rocprofv3 kernel-trace + stats of the config-3 training step (bench.py --train), no PMC.
# MODEL_ARGS='--embed_dim 256 --mha_heads 8': another model's step (bench.py --model-args).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/prof_train}
mkdir -p $P
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- \
  python bench.py --train --batch 8 --steps ${PROF_STEPS:-4} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} \
  ${MODEL_ARGS:+--model-args "$MODEL_ARGS"} > $P/bench_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 $P/bench_prof.log
find $P -name "*stats*" | head
exit $rc
