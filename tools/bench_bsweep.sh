set -u
mkdir -p gpurun_out
for b in 4 8 16 32; do
timeout -k 10 300 python -u bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_b$b.log 2>&1 || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_b$b.log').read().strip().splitlines()[-1]);print($b, d['value'], d['us_per_denoise_step'], d['roofline']['avg_launch_us'], d['roofline_attn_temporal']['avg_launch_us'])"
done
