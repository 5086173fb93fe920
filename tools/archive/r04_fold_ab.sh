#!/bin/bash
# MFMA fold build variants (tools/bin_fold_<v>, fold_bench.hip with -D flags)
# at B = 64 / 128 / 256, interleaved over 2 rounds.   tools/r04_fold_ab.sh <tag> <v>...
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/$1"; shift
mkdir -p "$OUT"
for r in 1 2; do
  for b in ${FOLD_BS:-64 128 256}; do
    for v in "$@"; do
      FOLD_MODE=mfma timeout -k 10 120 tools/bin_fold_$v $b 32 24 > "$OUT/tmp.json" 2>> "$OUT/err.log"
      rc=$?; [ $rc -le 1 ] || { echo "$v $b rc=$rc"; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/tmp.json')); print('$v', '$b', 'r$r', d['fold_us'], d['ok'])" | tee -a "$OUT/ab.txt"
    done
  done
done
