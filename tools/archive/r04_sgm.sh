#!/bin/bash
# MFMA fold: key-major selection bits (EvalFull's layout) vs super-group-major.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04sgm}"
mkdir -p "$OUT"
for r in 1 2; do
  for b in ${SGM_BS:-16 32 64 128 256}; do
    for g in 0 1 4; do
      FOLD_MODE=mfma FOLD_SGM=$g timeout -k 10 120 tools/fold_bench $b 32 24 > "$OUT/tmp.json" 2>> "$OUT/err.log"
      rc=$?; [ $rc -le 1 ] || { echo "sgm$g $b rc=$rc"; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/tmp.json')); print('sgm$g', '$b', 'r$r', d['fold_us'], d['ok'])" | tee -a "$OUT/ab.txt"
    done
  done
done
