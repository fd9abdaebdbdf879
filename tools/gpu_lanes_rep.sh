set -u
cd "${GRAFT_REPO_ROOT}"
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "concurrent_lanes" -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1
done
