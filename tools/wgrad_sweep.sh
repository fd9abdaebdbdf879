#!/bin/bash
# wgrad microbench under ring depths (MDG_WGRAD_STAGES) x split targets (MDG_WGRAD_BLOCKS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for ns in 3 4 5; do
  for nb in 512 768 1024; do
    echo "== stages $ns blocks $nb"
    MDG_WGRAD_STAGES=$ns MDG_WGRAD_BLOCKS=$nb timeout -k 10 120 python tools/wgrad_bench.py 2>&1 | grep -v amdgpu.ids | cut -c1-70 || exit $?
  done
done
