#!/bin/bash
# Interleaved A/B of library builds on one bench workload (default eval).
# Usage: tools/r06_ab_eval.sh <rounds> <lib.so|product> ...   env WL=eval|pir|split
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
R=$1; shift
WL="${WL:-eval}"
for r in $(seq 1 "$R"); do
  for L in "$@"; do
    if [ "$L" = product ]; then E=(); else E=(env "DPF_LIB=$REPO/$L"); fi
    out=$("${E[@]}" timeout -k 10 120 python bench.py --workload "$WL" --steps 20 --warmup 5 --no-cpu-baseline --no-sweep ${EXTRA:-} 2>/dev/null | grep '^{') || { echo "FAIL $L"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$L', d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
  done
done
