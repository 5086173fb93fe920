#!/bin/bash
# r05: the fold at 2 workgroups per CU for cached slices and <= 32 keys:
# the fold / PIR / per-rank GPU tests, then fold_bench and the PIR step.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fpercu2}"; mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fold.py \
   tests/test_gpu_per_rank.py tests/test_gpu_pir.py tests/test_gpu_pir_fused.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
export FOLD_MODE=mfma
for r in 1 2 3; do
  for cfg in "16 32 24" "32 32 24" "64 32 24" "64 32 23" "64 32 22" "64 32 21"; do
    timeout -k 10 60 tools/fold_bench $cfg > "$OUT/fb.json" 2>&1 || { echo "fold_bench $cfg failed"; cat "$OUT/fb.json"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r $cfg', d['fold_us'], 'us ok', d['ok'])" | tee -a "$OUT/fold.txt"
  done
done
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads --workload pir"
for r in 1 2 3; do
  for W in 1 4 8; do
    timeout -k 10 120 python3 bench.py $C --emulate-world $W > "$OUT/pir.log" 2>&1 || { echo "FAIL pir"; tail -3 "$OUT/pir.log"; exit 1; }
    grep '^{' "$OUT/pir.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r W=$W', round(d['ms_per_step'],4))" | tee -a "$OUT/pir.txt"
  done
done
