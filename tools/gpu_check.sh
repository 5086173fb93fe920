#!/bin/bash
# One GPU-box session: parity tests, then every bench workload with --check.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-check}"
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
for w in evalfull eval split pir; do
  timeout -k 10 300 python bench.py --workload $w --check --steps 30 --warmup 10 --cpu-seconds 10 > "$OUT/bench_$w.log" 2>&1
  rc=$?; echo "bench $w rc=$rc"; grep '^{' "$OUT/bench_$w.log" | tail -1
  [ $rc -eq 0 ] || exit $rc
done
