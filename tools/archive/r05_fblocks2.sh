#!/bin/bash
# r05: 2 vs 3 fold workgroups per CU (512 vs 768 on 256 CUs) at B = 64 over
# 2^21 .. 2^24 records and B = 16 / 256 at 2^24, interleaved, 5 runs.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fblocks2}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for r in 1 2 3 4 5; do
  for cfg in "64 32 21" "64 32 22" "64 32 23" "64 32 24" "16 32 24" "256 32 24" "32 32 24"; do
    for nb in 512 768; do
      FOLD_BLOCKS=$nb timeout -k 10 60 tools/fold_bench $cfg > "$OUT/fb.json" 2>&1 || { echo "fold_bench $nb $cfg failed"; cat "$OUT/fb.json"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r $cfg blocks<=$nb', d['fold_us'], 'us ok', d['ok'])" | tee -a "$OUT/fblocks.txt"
    done
  done
done
