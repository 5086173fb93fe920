#!/bin/bash
# configs[1] strong scaling per-rank shapes (4096 keys over W = 1, 2, 4, 8
# emulated ranks) with the default sampled kernel events, plus the headline.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04strong}"
mkdir -p "$OUT"
B=(--steps 200 --warmup 20 --no-cpu-baseline --no-variants --no-api --no-workloads)
run() {   # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py "${B[@]}" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; [ $rc -le 1 ] || { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), r.get('kernel_ms'), round(d['value']/1e12,4))"
}
for r in 1 2 3; do
  for w in 1 2 4 8; do run "strong${w}_$r" --strong --nkeys 4096 --emulate-world $w; done
done
run full_check --check
