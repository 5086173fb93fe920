#!/bin/bash
# r05: persistent batched Eval, second form (stores issued after the slot
# wait) vs k_eval2 at configs[2]; Eval parity tests with it first.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_persist2}"; mkdir -p "$OUT"
export TMPDIR=/tmp
DPF_EVAL_PERSIST=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
   tests/test_gpu_eval_configs.py tests/test_gpu_parity.py -k "eval or config2" > "$OUT/tests.log" 2>&1 \
   || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
B="--workload eval --steps 40 --warmup 5 --no-cpu-baseline"
for round in 1 2 3; do
  for u in 1 0; do
    DPF_EVAL_PERSIST=$u timeout -k 10 120 python3 bench.py $B > "$OUT/eval_p${u}_$round.log" 2>&1 || { echo "bench p=$u failed"; tail -5 "$OUT/eval_p${u}_$round.log"; exit 1; }
    grep '^{' "$OUT/eval_p${u}_$round.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('persist=$u round $round', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G q/s kernel', d['roofline']['kernel_ms'])" | tee -a "$OUT/ab.txt"
  done
done
