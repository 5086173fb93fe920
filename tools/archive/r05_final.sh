#!/bin/bash
# r05 final: the round profile (tools/archive/r05_round.sh) on the final code, then
# the per-rank shares of the strong-scaling splits at N = 4 / 8 (emulated
# rank 0) for DESIGN.md §7.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG="${1:-r05_final}"
bash tools/archive/r05_round.sh "$TAG" || exit 1
OUT="gpurun_out/$TAG"
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
for r in 1 2; do
  for s in "--workload pir --emulate-world 1" "--workload pir --emulate-world 4" "--workload pir --emulate-world 8" \
           "--workload split --emulate-world 8" "--strong --nkeys 4096 --emulate-world 8" "--workload split --emulate-world 1"; do
    timeout -k 10 120 python3 bench.py $C $s > "$OUT/rank.log" 2>&1 || { echo "FAIL $s"; tail -3 "$OUT/rank.log"; exit 1; }
    grep '^{' "$OUT/rank.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$s', round(d['ms_per_step'],4))" | tee -a "$OUT/ranks.txt"
  done
done
