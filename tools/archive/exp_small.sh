set -o pipefail
mkdir -p gpurun_out/small
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_small_calls.py tests/test_gpu_api.py tests/test_gpu_parity.py > gpurun_out/small/tests.log 2>&1 || { tail -30 gpurun_out/small/tests.log; exit 1; }
tail -2 gpurun_out/small/tests.log
timeout -k 10 300 python tools/small_calls.py > gpurun_out/small/small_calls.json || exit 1
cat gpurun_out/small/small_calls.json
for n in 12 16 20 21 22; do for m in 2 1; do
  timeout -k 10 120 tools/small_call_bench $n $m >> gpurun_out/small/c_level.jsonl || exit 1
done; done
cat gpurun_out/small/c_level.jsonl
