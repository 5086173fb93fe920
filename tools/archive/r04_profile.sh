#!/bin/bash
# r04 round profile (after tools/gpu_round.sh): the default bench under
# rocprofv3 kernel-trace + PMC passes (tools/profile.sh), kernel traces and
# PMC passes of the eval / split / pir lines, per-launch HBM traffic.
#   tools/r04_profile.sh <tag>     -> gpurun_out/<tag>/...
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
T="${1:-r04prof}"
mkdir -p "gpurun_out/$T"
bash tools/profile.sh "gpurun_out/$T/prof" > "gpurun_out/$T/profile.log" 2>&1 || { tail -20 "gpurun_out/$T/profile.log"; exit 1; }
echo "default profile done"
export TMPDIR=/tmp
for w in eval split pir; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/$T/kt_$w" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" --workload $w --steps 20 --warmup 5 --no-sweep > "$REPO/gpurun_out/$T/kt_$w.log" 2>&1 ) || { echo "kt $w failed"; exit 1; }
  echo "kt $w done"
done
for w in eval split pir; do
  bash tools/counters.sh "gpurun_out/$T/pmc_$w" $w > /dev/null 2>&1 || { echo "pmc $w failed"; exit 1; }
  python3 tools/traffic.py "gpurun_out/$T/pmc_$w/summary.json" "gpurun_out/$T/traffic_$w.json" > /dev/null
  echo "pmc $w done"
done
{ command -v go && go version; } > "gpurun_out/$T/go_probe.txt" 2>&1 || echo "go: not found on the GPU box ($(date -u +%FT%TZ))" > "gpurun_out/$T/go_probe.txt"
# Keep summaries, drop the per-dispatch CSVs (gpurun copies back at most 64 MiB).
find "gpurun_out/$T" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" -o -name "*agent_info.csv" \) -delete
du -sh "gpurun_out/$T"
echo "round profile done"
