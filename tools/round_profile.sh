#!/bin/bash
# End-of-milestone GPU pass: parity tests + the 4 bench lines (tools/gpu_round.sh),
# the default bench under rocprofv3 kernel-trace + PMC passes (tools/profile.sh),
# kernel traces of the secondary workloads, and the Go toolchain probe.
#   tools/round_profile.sh <tag>     -> gpurun_out/<tag>/...
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
T="${1:-round}"
bash tools/gpu_round.sh "$T" || exit $?
bash tools/profile.sh "gpurun_out/$T/prof" > "gpurun_out/$T/profile.log" 2>&1 || { tail -20 "gpurun_out/$T/profile.log"; exit 1; }
export TMPDIR=/tmp
for w in eval split pir; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$REPO/gpurun_out/$T/kt_$w" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" --workload $w --steps 20 --warmup 5 --no-sweep > "$REPO/gpurun_out/$T/kt_$w.log" 2>&1 ) || { echo "kt $w failed"; exit 1; }
done
for w in eval split pir; do
  bash tools/counters.sh "gpurun_out/$T/pmc_$w" $w > /dev/null 2>&1 || { echo "pmc $w failed"; exit 1; }
  python3 tools/traffic.py "gpurun_out/$T/pmc_$w/summary.json" "gpurun_out/$T/traffic_$w.json" > /dev/null
done
( cd /tmp && timeout -k 10 60 rocprofv3 -L > "$REPO/gpurun_out/$T/pmc_avail.txt" 2>&1 ) || true
# Instruction-cache behaviour of the headline kernel (its hot loop is ~30 KiB of code).
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d "$REPO/gpurun_out/$T/pmc_icache" \
    -o p --output-format csv -- python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-api --no-variants \
    > "$REPO/gpurun_out/$T/pmc_icache.log" 2>&1 ) || echo "icache pass failed (see pmc_icache.log)"
{ command -v go && go version; } > "gpurun_out/$T/go_probe.txt" 2>&1 || echo "go: not found on the GPU box ($(date -u +%FT%TZ))" > "gpurun_out/$T/go_probe.txt"
# gpurun copies back at most 64 MiB: keep the summaries, drop raw per-dispatch
# CSVs (counter_collection / kernel_trace rows) once they have been summarised.
find "gpurun_out/$T" -type f -size +2M -printf '%s %p\n' > "gpurun_out/$T/pruned_files.txt"
find "gpurun_out/$T" -type f -size +2M -delete
echo "round profile done"
