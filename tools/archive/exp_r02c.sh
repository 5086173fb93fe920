set -uo pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c/gpu_tests.log 2>&1 || { tail -20 gpurun_out/r02c/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02c/gpu_tests.log
for w in 5 5 60; do
timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-api > gpurun_out/r02c/def_w$w.log 2>&1 || exit 1
grep '^{' gpurun_out/r02c/def_w$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('warmup $w', round(d['ms_per_step'],4), r['kernel_ms'], d['aes_variants'])"
done
for impl in ttable bitsliced; do
timeout -k 10 200 python bench.py --workload pir --aes $impl --steps 20 --warmup 10 --check > gpurun_out/r02c/pir_$impl.log 2>&1 || exit 1
grep '^{' gpurun_out/r02c/pir_$impl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('pir $impl', round(d['ms_per_step'],4), r['kernel_ms'])"
done
