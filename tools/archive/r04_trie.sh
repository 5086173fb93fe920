#!/bin/bash
# Trie Eval (DPF_EVAL_TRIE=1) vs frontier + per-query walks, interleaved, configs[2].
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04trie}"
mkdir -p "$OUT"
B=(--workload eval --steps 30 --warmup 5 --no-cpu-baseline --no-variants --no-api --no-workloads)
run() {   # name trie args...
  local name=$1 tr=$2; shift 2
  DPF_EVAL_TRIE=$tr timeout -k 10 200 python bench.py "${B[@]}" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; [ $rc -le 1 ] || { echo "$name rc=$rc"; tail -5 "$OUT/$name.log"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), r.get('kernel_ms'), round(d['value']/1e9,3))"
}
run trie_check 1 --check
for r in 1 2; do
  run "walk_$r" 0
  run "trie_$r" 1
done
