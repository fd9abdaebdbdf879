#!/bin/bash
# Same-box A/B timing, one script for every kind (replaces ab_env / ab_env_train / ab_infer /
# ab_micro / ab_train / gpu_ab / gpu_ab_env).  Variants alternate, AB_REPS (2) rounds, so box drift
# hits both alike.  Two variants, A and B, each an environment setting ("" = none); B may also be
# the library ablib/old.so (tools/build_ab.sh) by AB_B_LIB=1.
#   AB_WHAT=infer  the bench line (frames/s, us per denoise step, roofline kernels' live us)
#   AB_WHAT=train  the --train line (ms per step)
#   AB_WHAT=micro  AB_MICRO="script args" (a microbenchmark; its last AB_LINES lines)
# AB_TESTS (a pytest -k filter over the kernel / parity / training tests) runs once per variant
# first and stops the script on a failure.
#   AB_WHAT=train AB_A="" AB_B="MDG_ATTN_BWD_FOLD=0" bash tools/ab.sh
#   AB_ARGS is evaluated: AB_ARGS="--model-args '--embed_dim 256 --mha_heads 8'" passes one argument
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WHAT=${AB_WHAT:-infer}
run_variant() {  # $1 = A | B
  local V=$1 E
  if [ "$V" = A ]; then E=${AB_A:-}; else E=${AB_B:-}; fi
  if [ "$V" = B ] && [ "${AB_B_LIB:-0}" = 1 ]; then E="$E MDG_LIB_PATH=$PWD/ablib/old.so"; fi
  case $WHAT in
  infer)
    eval "env $E timeout -k 10 300 python -u bench.py --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline --no-f32-line \
      --sweep-batches '' ${AB_ARGS:-}" > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || { tail -5 gpurun_out/ab_$V.err; return 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$V.json') if l.startswith('{')][-1]);print('$V [$E]', d['value'], d['us_per_denoise_step'], [r['avg_launch_us'] for r in [d['roofline']]+(d['roofline_more'] or [])] if d.get('roofline') else '')" ;;
  train)
    eval "env $E timeout -k 10 300 python -u bench.py --train --batch 8 --steps ${AB_STEPS:-10} --warmup 2 --no-cpu-baseline \
      ${AB_ARGS:-}" > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || { tail -5 gpurun_out/ab_$V.err; return 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$V.json') if l.startswith('{')][-1]);print('$V [$E]', d['ms_per_step'], d['value'])" ;;
  micro)
    echo "== $V [$E]"; env $E timeout -k 10 120 python $AB_MICRO 2>&1 | grep -v amdgpu.ids | tail -${AB_LINES:-4} ;;
  esac
}
if [ -n "${AB_TESTS:-}" ]; then
  for V in A B; do
    if [ "$V" = A ]; then E=${AB_A:-}; else E=${AB_B:-}; fi
    env $E timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_train.py \
      -k "$AB_TESTS" -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab_$V.log 2>&1
    rc=$?; echo "tests $V rc=$rc"; tail -3 gpurun_out/pytest_ab_$V.log
    [ $rc -ne 0 ] && exit $rc
  done
fi
for rep in $(seq ${AB_REPS:-2}); do
  for V in A B; do run_variant $V || exit 1; done
done
