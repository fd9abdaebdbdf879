#!/bin/bash
# Quick GPU iteration: the GPU kernel + parity tests (-k filter via PYTEST_K), then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_quick.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_quick.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1]);print(d['value'], d['us_per_denoise_step'], [(r['kernel'], r['avg_launch_us']) for r in [d['roofline']]+d['roofline_more']])"
${EXTRA:+timeout -k 10 300 $EXTRA}
