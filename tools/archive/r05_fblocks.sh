#!/bin/bash
# r05: fold workgroup count at the per-rank DB slices (2^21 records: N = 8,
# 2^22: N = 4), B = 64: fewer workgroups mean fewer partials for
# k_xor_parts but less parallelism in the fold (FOLD_BLOCKS caps the grid).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fblocks}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for r in 1 2 3; do
  for lg in 21 22; do
    for nb in 128 256 384 512 1024; do
      FOLD_BLOCKS=$nb timeout -k 10 60 tools/fold_bench 64 32 $lg > "$OUT/fb.json" 2>&1 || { echo "fold_bench $nb $lg failed"; cat "$OUT/fb.json"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r logN=$lg blocks<=$nb', d['fold_us'], 'us ok', d['ok'])" | tee -a "$OUT/fblocks.txt"
    done
  done
done
