#!/bin/bash
# Round 4: TPS graphed-vs-eager diagnostic (library vs torch optimizer), full GPU suite, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "diag_tps|200|python -u tools/diag_tps_graph.py" \
  "gpusuite|1000|python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests" \
  "trainprof|200|bash tools/gpu_train_prof.sh"
