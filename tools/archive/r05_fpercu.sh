#!/bin/bash
# r05: fold workgroups per CU (DPF_FOLD_PER_CU caps the occupancy the
# launcher reads): the default against 2 per CU on tools/fold_bench at the
# configs[4] DB (B = 16, 32, 64) and the per-rank slices, then the PIR step at
# N = 1 / 4 / 8 (emulated rank 0), interleaved.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fpercu}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for r in 1 2 3 4 5; do
  for cfg in "16 32 24" "32 32 24" "64 32 24" "64 32 23" "64 32 22" "64 32 21"; do
    for pc in 0 2; do
      DPF_FOLD_PER_CU=$pc timeout -k 10 60 tools/fold_bench $cfg > "$OUT/fb.json" 2>&1 || { echo "fold_bench $pc $cfg failed"; cat "$OUT/fb.json"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r $cfg per_cu=$pc', d['fold_us'], 'us ok', d['ok'])" | tee -a "$OUT/fold.txt"
    done
  done
done
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads --workload pir"
for r in 1 2 3; do
  for W in 1 4 8; do
    for pc in 0 2; do
      DPF_FOLD_PER_CU=$pc timeout -k 10 120 python3 bench.py $C --emulate-world $W > "$OUT/pir.log" 2>&1 || { echo "FAIL pir"; tail -3 "$OUT/pir.log"; exit 1; }
      grep '^{' "$OUT/pir.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r W=$W per_cu=$pc', round(d['ms_per_step'],4))" | tee -a "$OUT/pir.txt"
    done
  done
done
