#!/bin/bash
# World-1 RCCL rehearsal of the graphed DDP step with bucket markers (MDG_BUCKET_MARK=1): the bench
# line (bucket sizes) and a rocprofv3 kernel trace, summarised by tools/rccl_overlap_trace.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PROF_DIR:-gpurun_out/prof_rehearsal}
mkdir -p $P
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export MDG_BUCKET_MARK=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- \
  python bench.py --train --batch 8 --steps 3 --warmup 2 --no-cpu-baseline --train-rccl1 ${BENCH_ARGS:-} > $P/bench.json 2> $P/bench.err
rc=$?; echo "prof rc=$rc"; tail -2 $P/bench.err
[ $rc -ne 0 ] && exit $rc
python - "$P" <<'PY'
import json, subprocess, sys
P = sys.argv[1]
d = json.loads(open(P + "/bench.json").read().strip().splitlines()[-1])
b = d["allreduce_buckets"]
print("ms/step", d["ms_per_step"], "buckets", b["n"], "bytes", b["bytes"], "replicated", d.get("replicated_conditioning_params"))
subprocess.check_call([sys.executable, "tools/rccl_overlap_trace.py", P + "/run_kernel_trace.csv", str(b["n"]),
                       P + "/overlap.md", ",".join(str(x) for x in b["bytes"])])
PY
