set -uo pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 120 ./tools/bin/gen_bench 20 16 400000 > gpurun_out/r02f/gen_bench.json 2>&1 || exit 1; cat gpurun_out/r02f/gen_bench.json
timeout -k 10 120 ./tools/bin/gen_bench 24 16 200000 > gpurun_out/r02f/gen_bench24.json 2>&1 || exit 1; cat gpurun_out/r02f/gen_bench24.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02f/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02f/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-api --no-variants > gpurun_out/r02f/bench_gpus2.log 2>&1; rc=$?; grep '^{' gpurun_out/r02f/bench_gpus2.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/r02f/bench_gpus2.log; exit $rc; }
