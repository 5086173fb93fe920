#!/bin/bash
# One GPU-box call: GPU parity tests, then the default bench line (driver
# command) and the secondary workloads.  Each step has its own time limit and
# the first failure ends the call.  Usage: tools/gpu_round.sh <tag> [pytest -k expr]
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-round}"
mkdir -p "$OUT"
K=()
[ $# -ge 2 ] && K=(-k "$2")
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
    > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_default.log" 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' "$OUT/bench_default.log" | tail -1
[ $rc -eq 0 ] || exit $rc
for w in eval split pir; do
  timeout -k 10 300 python bench.py --workload $w --check --steps 20 --warmup 5 > "$OUT/bench_$w.log" 2>&1
  rc=$?; echo "bench $w rc=$rc"; grep '^{' "$OUT/bench_$w.log" | tail -1
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"
exit $rc
