#!/bin/bash
# Profiles bench.py's EvalFull step with rocprofv3 on the GPU box:
#   1. --kernel-trace --stats (per-kernel durations)
#   2..n. PMC passes, each counter group in its own run (no tracing domains
#      combined with --pmc): FETCH_SIZE, WRITE_SIZE, SQ instruction mix.
# Usage: tools/profile.sh <out_dir> [extra bench.py args...]
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/${1:-gpurun_out/prof}"
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline "$@")

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${BENCH[@]}" \
    > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- "${BENCH[@]}" \
    > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- "${BENCH[@]}" \
    > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d "$OUT/sq" -o sq --output-format csv -- "${BENCH[@]}" > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
    -d "$OUT/lds" -o lds --output-format csv -- "${BENCH[@]}" > "$OUT/lds.log" 2>&1
echo "profile done: $OUT"
