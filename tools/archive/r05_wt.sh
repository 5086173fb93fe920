#!/bin/bash
# r05: per-wave timing of the tree kernel at the small per-rank shapes, with
# the root-to-subtree walk's end (tools/wave_times.hip, built in tools/bin):
# how much of a launch is the serial walk.  Shapes: "nkeys logN prefix_bits".
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_wt}"; mkdir -p "$OUT"
for shape in "64 24 3" "64 24 2" "64 24 0" "1 32 3" "512 20 0" "4096 20 0"; do
  tag=${shape// /_}
  WAVE_TIMES_CSV="$OUT/wt_$tag.csv" timeout -k 10 120 tools/bin/wave_times $shape >> "$OUT/wt.jsonl" || { echo "wt $shape failed"; exit 1; }
  tail -1 "$OUT/wt.jsonl"
done
gzip -f "$OUT"/*.csv
