#!/bin/bash
# Lane-divergence locus hunt (tools/lane_race.py), one process per variant.
# Round-3 results: gpurun_out/lane_race/*.log; DESIGN.md §2 records the cause.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/lane_race
mkdir -p $OUT
R=${R:-300}
run() { local name=$1; shift; echo "== $name"; env "$@" timeout -k 10 150 python -u tools/lane_race.py $LA > $OUT/$name.log 2>&1; local rc=$?; tail -1 $OUT/$name.log; return $rc; }
VARIANTS=${VARIANTS:-"default spa3 spa4 xcd0 fence dppc nomlp"}
for v in $VARIANTS; do
  case $v in
    default) LA="3 1 $R" run default MDG_X=1 ;;
    spa3) LA="3 1 $R" run spa3 MDG_SPA_STAGES=3 ;;
    spa4) LA="3 1 $R" run spa4 MDG_SPA_STAGES=4 ;;
    xcd0) LA="3 1 $R" run xcd0 MDG_SPA_XCD=0 ;;
    fence) LA="3 1 $R" run fence MDG_LIB_PATH=$PWD/diaglib/spa1.so ;;
    dppc) LA="3 1 $R" run dppc MDG_LIB_PATH=$PWD/diaglib/spa2.so ;;
    nomlp) LA="3 1 $R" run nomlp MDG_FUSED_MLP=0 ;;
    acq) LA="3 1 $R" run acq MDG_LIB_PATH=$PWD/diaglib/spa3.so ;;
    sys) LA="3 1 $R" run sys MDG_LIB_PATH=$PWD/diaglib/spa4.so ;;
    areg) LA="3 1 $R" run areg MDG_LIB_PATH=$PWD/diaglib/spa5.so ;;
    sleep) LA="3 1 $R" run sleep MDG_LIB_PATH=$PWD/diaglib/spa6.so ;;
    twice) LA="3 1 $R" run twice MDG_LIB_PATH=$PWD/diaglib/spa9.so ;;
    vh) LA="3 1 $R" run vh MDG_LIB_PATH=$PWD/diaglib/vh.so ;;
    vT) LA="3 1 $R" run vT MDG_LIB_PATH=$PWD/diaglib/vT.so ;;
    vP) LA="3 1 $R" run vP MDG_LIB_PATH=$PWD/diaglib/vP.so ;;
    vX) LA="3 1 $R" run vX MDG_LIB_PATH=$PWD/diaglib/vX.so ;;
    o2) LA="3 2 $R" run o2 MDG_X=1 ;;
    l2o1) LA="2 1 $R 4" run l2o1 MDG_X=1 ;;
    vR) LA="3 1 $R" run vR MDG_LIB_PATH=$PWD/diaglib/vR.so ;;
    order) LA="3 1 $R" run order MDG_LIB_PATH=$PWD/diaglib/order.so ;;
    *) echo "unknown $v"; false ;;
  esac || exit 1
done
