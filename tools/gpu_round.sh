#!/bin/bash
# Full round evidence on one box: smoke + GPU tests + bench (gpu_check.sh), then the rocprofv3
# kernel-trace/stats pass (gpu_prof.sh), then the FETCH_SIZE / WRITE_SIZE PMC passes
# (roof_pmc.sh).  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh || exit $?
bash tools/gpu_prof.sh || exit $?
bash tools/roof_pmc.sh || exit $?
