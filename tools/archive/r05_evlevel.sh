#!/bin/bash
# r05: batched Eval frontier one level deeper (DPF_EVAL_LEVEL_SHIFT=1: L = 10
# at configs[2], 2046 + 4 x 1024 blocks per key instead of 1022 + 5 x 1024),
# interleaved with the product level, plus --check on each.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_evlevel}"; mkdir -p "$OUT"
for r in 1 2 3; do
  for sh in 0 1; do
    DPF_EVAL_LEVEL_SHIFT=$sh timeout -k 10 180 python3 bench.py --workload eval --steps 40 --warmup 8 --no-cpu-baseline \
        --no-api $( [ $r = 1 ] && echo --check ) > "$OUT/run.log" 2>&1 || { echo "shift $sh failed"; tail -5 "$OUT/run.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); print('$r shift $sh', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G q/s')" | tee -a "$OUT/ab.txt"
  done
done
