#!/bin/bash
# PIR workload: bench line plus per-kernel times (rocprofv3 kernel trace).
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/${1:-pirprof}"; shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --workload pir --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
grep '^{' "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'])"
cut -d, -f1-8 "$OUT/kt/kt_kernel_stats.csv"
