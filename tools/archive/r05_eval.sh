#!/bin/bash
# r05: the L2-scratch trie Eval kernel (k_eval_trie) vs frontier + walks
# (k_eval2) at configs[2]: parity tests, interleaved bench lines, kernel trace.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_eval}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_eval_configs.py \
   > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
B="--workload eval --steps 40 --warmup 5 --no-cpu-baseline"
for round in 1 2 3; do
  for t in 0 1; do
    DPF_EVAL_TRIE=$t timeout -k 10 120 python3 bench.py $B > "$OUT/eval_t${t}_$round.log" 2>&1 || { echo "bench trie=$t failed"; tail -5 "$OUT/eval_t${t}_$round.log"; exit 1; }
    grep '^{' "$OUT/eval_t${t}_$round.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('trie=$t round $round', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G q/s kernel', d['roofline']['kernel_ms'])"
  done
done
for t in 0 1; do
  ( cd /tmp && DPF_EVAL_TRIE=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_t$t" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" $B > "$REPO/$OUT/kt_t$t.log" 2>&1 ) || { echo "kt $t failed"; exit 1; }
  python3 - "$REPO/$OUT/kt_t$t" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(" ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
