#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters in this pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/prof}
mkdir -p $P
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- \
  python bench.py --steps ${PROF_STEPS:-3} --warmup 1 --no-cpu-baseline --sweep-batches "" --no-f32-line ${BENCH_ARGS:-} > $P/bench_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 $P/bench_prof.log
find $P -name "*stats*" | head
exit $rc
