set -uo pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_pir.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02e/fold_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r02e/fold_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/bin/gen_bench 20 16 400000 > gpurun_out/r02e/gen_bench.json 2>&1; cat gpurun_out/r02e/gen_bench.json
timeout -k 10 120 ./tools/bin/gen_bench 24 16 200000 > gpurun_out/r02e/gen_bench24.json 2>&1; cat gpurun_out/r02e/gen_bench24.json
