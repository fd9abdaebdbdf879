#!/bin/bash
# Same-box A/B of a microbench (python script + args) under the tree's library and ablib/old.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export MDG_LIB_PATH=$PWD/ablib/old.so; else unset MDG_LIB_PATH; fi
    echo "== $L"; timeout -k 10 120 python "$@" 2>&1 | grep -v amdgpu.ids | tail -${AB_LINES:-4} || exit $?
  done
done
