#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters in this pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps ${PROF_STEPS:-3} --warmup 1 --no-cpu-baseline --sweep-batches "" --no-f32-line ${BENCH_ARGS:-} > gpurun_out/prof/bench_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/prof/bench_prof.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
