#!/bin/bash
# A/B of library builds on the default bench workload, interleaved rounds.
# Usage: tools/ab_libs.sh <rounds> <lib1.so> <lib2.so> ... (paths relative to repo)
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
R=$1; shift
for r in $(seq 1 $R); do
  for L in "$@"; do
    out=$(DPF_LIB="$REPO/$L" timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-api ${AB_ARGS:-} 2>/dev/null | grep '^{') || { echo "FAIL $L"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); v=d.get('aes_variants',{}); print('$r', '$L', round(d['value']/1e12,4), d['roofline']['kernel_ms'], {k: round(x['kernel_ms'],4) for k,x in v.items()})"
  done
done
