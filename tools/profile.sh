#!/bin/bash
# Round profile of the exact driver bench command (python bench.py, defaults):
#   1. rocprofv3 --kernel-trace --stats around `python3 bench.py` (its JSON
#      line is kept beside the stats, so the kernel averages can be compared
#      with the line's roofline.kernel_ms)
#   2. PMC passes (each counter group alone) on a short bench run, then
#      per-launch HBM traffic via tools/traffic.py
# Usage: tools/profile.sh <out_dir>
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/${1:-gpurun_out/prof}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" > "$OUT/bench_under_rocprof.log" 2>&1
grep '^{' "$OUT/bench_under_rocprof.log" > "$OUT/bench_line.json"
cp "$OUT/kt/kt_kernel_stats.csv" "$OUT/kernel_stats.csv"
"$REPO/tools/counters.sh" "${1:-gpurun_out/prof}/pmc" evalfull > /dev/null
python3 "$REPO/tools/traffic.py" "$OUT/pmc/summary.json" "$OUT/traffic.json"
echo "profile done: $OUT"
