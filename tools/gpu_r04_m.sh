#!/bin/bash
# Round 4: TPS graphed-vs-eager diagnostic; the graphed-step tests with thread-local capture.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "diag_tps|200|python -u tools/diag_tps_graph.py" \
  "graphtests|400|python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_train.py -k 'graphed or world2 or resume'"
