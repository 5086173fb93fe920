#!/bin/bash
# r06: matrix-core fold variants (tools/bin/fold_<v>, fold_bench.hip built with
# -D flags) at B = 64 over 2^24 x 32 B, interleaved rounds.  Args: <out> <v>...
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/$1"; shift
mkdir -p "$OUT"
for r in 1 2 3; do
  for b in ${FOLD_BS:-64}; do
    for v in "$@"; do
      FOLD_MODE=mfma timeout -k 10 120 tools/bin/fold_$v $b 32 ${FOLD_LOGN:-24} > "$OUT/tmp.json" 2>> "$OUT/err.log"
      rc=$?; [ $rc -le 1 ] || { echo "$v $b rc=$rc"; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/tmp.json')); print('$v', '$b', 'r$r', d['fold_us'], d['ok'])" | tee -a "$OUT/ab.txt"
    done
  done
done
