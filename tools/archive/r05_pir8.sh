#!/bin/bash
# configs[4] per-rank share at N = 4 and 8 (emulated on one GPU) on the r04+
# product path (sliced MFMA fold, keys read in place): bench lines, subtree
# depth sweep, and a rocprofv3 kernel trace of each shape.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_pir8}"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="--workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep"
for W in 1 4 8; do
  timeout -k 10 120 python3 bench.py $B --emulate-world $W > "$OUT/pir_w$W.log" 2>&1 || { echo "bench W=$W failed"; tail -5 "$OUT/pir_w$W.log"; exit 1; }
  grep '^{' "$OUT/pir_w$W.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('W=$W step', round(d['ms_per_step'],4), 'tree', k['tree']['kernel_ms'], 'fold', k['fold']['kernel_ms'], 'b2b', k['back_to_back'])"
done
for W in 8; do
  for D in 1 2 3 4 5; do
    DPF_SUBTREE_DEPTH=$D timeout -k 10 120 python3 bench.py $B --emulate-world $W > "$OUT/pir_w${W}_d$D.log" 2>&1 || { echo "bench W=$W D=$D failed"; exit 1; }
    grep '^{' "$OUT/pir_w${W}_d$D.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('W=$W D=$D step', round(d['ms_per_step'],4), 'tree', k['tree']['kernel_ms'], 'fold', k['fold']['kernel_ms'])"
  done
done
for W in 4 8; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_w$W" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" $B --emulate-world $W > "$REPO/$OUT/kt_w$W.log" 2>&1 ) || { echo "kt W=$W failed"; exit 1; }
  python3 - "$REPO/$OUT/kt_w$W" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(" ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
