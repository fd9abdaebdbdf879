#!/bin/bash
# GPU evidence steps by name, one parameterised script for every round (replaces the per-round
# gpu_r0*_*.sh launchers).  Each step runs under its own limit through tools/gpu_steps.sh, which
# stops at a crash / abort / timeout.  Outputs: gpurun_out/r${ROUND}_<step>.{log,json}.
# usage: ROUND=06 tools/evidence.sh step [step ...]      (a quoted "name|secs|cmd" runs as is)
#   smoke     __graft_entry__.smoke()
#   suite     the GPU test suite (tools/gpu_suite.sh; parity errors logged)
#   bench     the default bench line (BASELINE config 2)            prof      its kernel trace
#   roofpmc   PMC traffic / SQ passes of the bench roofline kernels
#   b1        the reference's sim_inference shape (B = 1, one lane)  prof_b1   its kernel trace
#   split     sim_inference over a peptide split, serial vs batched (tools/split_bench.py)
#   tps       TPS B = 16 x T = 100 (config 4)                       atlas     ATLAS T = 250 x crop 256 (config 5)
#   train     config 3's training step, B = 8 x T = 1000            trainprof its kernel trace
#   trainpmc  PMC / SQ passes of the training step
#   rccl1     the training step with a world-1 RCCL group (in-graph bucket all-reduces + cond all-gathers)
#   share2    bench.py --gpus 2 with both ranks on cuda:0 (the N-GPU launch path rehearsed; gloo)
#   share2tr  the same under torch.distributed.run (the driver's N-GPU launch form)
#   dopri5    the reference's default sampler
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${ROUND:-06}
declare -A S=(
  [smoke]="r${R}_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'"
  [suite]="r${R}_suite|960|bash tools/gpu_suite.sh"
  [bench]="r${R}_bench|400|python bench.py > gpurun_out/r${R}_bench.json"
  [prof]="r${R}_prof|300|bash tools/gpu_prof.sh"
  [roofpmc]="r${R}_roofpmc|400|bash tools/roof_pmc.sh"
  [b1]="r${R}_b1|200|python bench.py --batch 1 --lanes 1 --steps 3 --warmup 1 --sweep-batches '' --no-f32-line > gpurun_out/r${R}_bench_b1.json"
  [prof_b1]="r${R}_prof_b1|200|PROF_DIR=gpurun_out/prof_b1 BENCH_ARGS='--batch 1 --lanes 1' bash tools/gpu_prof.sh"
  [split]="r${R}_split|300|python tools/split_bench.py > gpurun_out/r${R}_split.json"
  [tps]="r${R}_tps|200|python bench.py --tps --frames 100 --batch 16 --steps 3 --warmup 1 --sweep-batches '' --no-f32-line > gpurun_out/r${R}_bench_tps.json"
  [atlas]="r${R}_atlas|400|python bench.py --frames 250 --crop 256 --batch 1 --lanes 1 --steps 3 --warmup 1 --sweep-batches '' --no-f32-line --cpu-seconds 20 > gpurun_out/r${R}_bench_atlas.json"
  [train]="r${R}_train|300|python bench.py --train --batch 8 > gpurun_out/r${R}_bench_train.json"
  [trainprof]="r${R}_trainprof|300|bash tools/gpu_train_prof.sh"
  [trainpmc]="r${R}_trainpmc|400|bash tools/train_pmc.sh"
  [rccl1]="r${R}_rccl1|300|python bench.py --train --train-rccl1 --batch 8 --no-cpu-baseline > gpurun_out/r${R}_bench_rccl1.json"
  [share2]="r${R}_share2|400|MDG_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r${R}_share2.json"
  [share2tr]="r${R}_share2tr|400|MDG_BENCH_SHARE_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r${R}_share2tr.json"
  [dopri5]="r${R}_dopri5|200|python bench.py --sampler dopri5 --steps 2 --warmup 1 > gpurun_out/r${R}_bench_dopri5.json"
)
args=()
for n in "$@"; do
  if [ -n "${S[$n]:-}" ]; then args+=("${S[$n]}"); else args+=("$n"); fi
done
bash tools/gpu_steps.sh "${args[@]}"
