#!/bin/bash
# r05: nontemporal DB loads in k_fold_mfma by DB size (DPF_FOLD_NT_MIN=0:
# always, 1<<62: never) at B = 64 over 2^21..2^24 records of 32 B, and
# B = 16 / 256 at 2^24; then the PIR step (1 GPU and the N = 8 / 4 ranks).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_nt}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for r in 1 2 3; do
  for cfg in "64 32 21" "64 32 22" "64 32 23" "64 32 24" "1 32 24" "16 32 24" "256 32 24"; do
    for nt in 0 4611686018427387904; do
      DPF_FOLD_NT_MIN=$nt timeout -k 10 60 tools/fold_bench $cfg > "$OUT/fb.json" 2>&1 || { echo "fold_bench $cfg failed"; cat "$OUT/fb.json"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r $cfg nt=' + ('always' if '$nt' == '0' else 'never'), d['fold_us'], 'us', d['GBs'], 'GB/s ok', d['ok'])" | tee -a "$OUT/nt.txt"
    done
  done
done
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads --workload pir"
for r in 1 2; do
  for W in 1 4 8; do
    for nt in 0 4611686018427387904; do
      DPF_FOLD_NT_MIN=$nt timeout -k 10 120 python3 bench.py $C --emulate-world $W > "$OUT/pir.log" 2>&1 || { echo "FAIL pir"; tail -3 "$OUT/pir.log"; exit 1; }
      grep '^{' "$OUT/pir.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r W=$W nt=' + ('always' if '$nt' == '0' else 'never'), round(d['ms_per_step'],4), 'fold', d.get('breakdown',{}).get('back_to_back',{}).get('fold_ms'))" | tee -a "$OUT/pir.txt"
    done
  done
done
