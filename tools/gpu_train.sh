set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train.log 2>&1; rc=$?
echo "train test rc=$rc"; tail -5 gpurun_out/pytest_train.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/train_bench.py --batch 8 --steps 4 --warmup 2 > gpurun_out/train_bench_fp32.log 2>&1; rc=$?
echo "train fp32 rc=$rc"; tail -3 gpurun_out/train_bench_fp32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/train_bench.py --batch 8 --steps 4 --warmup 2 --precision bf16-mixed > gpurun_out/train_bench_bf16.log 2>&1; rc=$?
echo "train bf16 rc=$rc"; tail -3 gpurun_out/train_bench_bf16.log
exit $rc
