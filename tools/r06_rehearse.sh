#!/bin/bash
# r06: the driver's multi-GPU bench command rehearsed on the 1-GPU box (ranks
# folded onto cuda:0, gloo control plane; lines marked folded_ranks), N = 2
# and 8, with the final code.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r06_rehearse}"; mkdir -p "$OUT"
for n in 2 8; do
  timeout -k 10 400 python3 bench.py --gpus $n --steps 10 --warmup 3 > "$OUT/g$n.log" 2>&1 || { echo "gpus=$n failed"; tail -20 "$OUT/g$n.log"; exit 1; }
  grep '^{' "$OUT/g$n.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gpus=$n', d['n_gpus'], d.get('folded_ranks'), d['value'], d['ms_per_step'], sorted((d.get('workloads') or {}).keys()))" | tee -a "$OUT/rehearse.txt"
done
