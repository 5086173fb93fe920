set -uo pipefail
mkdir -p gpurun_out/r02m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02m/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02m/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-api --check > gpurun_out/r02m/bench_$i.log 2>&1 || exit 1
grep '^{' gpurun_out/r02m/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], round(d['ms_per_step'],4), r['kernel_ms'], d['aes_variants']['bitsliced']['bit_identical_first_64_keys'])"
done
