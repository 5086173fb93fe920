set -uo pipefail
mkdir -p gpurun_out/r02l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02l/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02l/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload eval --check --steps 20 --warmup 5 > gpurun_out/r02l/bench_eval.log 2>&1 || exit 1
grep '^{' gpurun_out/r02l/bench_eval.log | cut -c1-300
bash tools/counters.sh gpurun_out/r02l/pmc_eval eval > /dev/null 2>&1 && python3 tools/traffic.py gpurun_out/r02l/pmc_eval/summary.json gpurun_out/r02l/traffic_eval.json > /dev/null && python3 -c "
import json; t=json.load(open('gpurun_out/r02l/traffic_eval.json'))
[print(k, round(v['fetch_bytes']/1e6,1), round(v['write_bytes']/1e6,1), v['avg_ns']) for k,v in t.items() if k.startswith('k_')]"
