#!/bin/bash
# r05 end of round: the GPU suite, smoke() and the driver's default bench
# command on the final code.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_final2}"; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
t0=$(date +%s)
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.log" 2>&1
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - t0 ))s"; [ $rc -eq 0 ] || exit $rc
grep '^{' "$OUT/bench_default.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], {k: (v['value'], v['ms_per_step']) for k, v in d['workloads'].items()})"
