#!/bin/bash
# Kernel trace of the configs[4] PIR step, matrix-core fold vs LDS fold.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04pirprof}"
mkdir -p "$OUT"
export TMPDIR=/tmp
for f in mfma lds; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_$f" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" --workload pir --pir-fold $f --steps 30 --warmup 5 --no-sweep --no-cpu-baseline \
      > "$REPO/$OUT/kt_$f.log" 2>&1 ); echo "kt $f rc=$?"
  python3 - "$REPO/$OUT/kt_$f/kt_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(" ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
  grep '^{' "$REPO/$OUT/kt_$f.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  step', d['ms_per_step'], d['kernels']['tree']['kernel_ms'], d['kernels']['fold']['kernel_ms'])"
done
