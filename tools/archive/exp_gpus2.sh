#!/bin/bash
# 2-rank rehearsal of bench.py --gpus 2 on a 1-GPU box (both ranks fold onto
# cuda:0, gloo control plane) for every workload, with --check.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-gpus2}"
mkdir -p "$OUT"
for w in ${WL:-evalfull split pir eval}; do
  timeout -k 10 300 python bench.py --gpus 2 --workload $w --steps 10 --warmup 3 --no-api --no-variants --no-cpu-baseline --check > "$OUT/$w.log" 2>&1
  rc=$?; grep '^{' "$OUT/$w.log" | cut -c1-300
  [ $rc -eq 0 ] || { tail -20 "$OUT/$w.log"; exit $rc; }
done
