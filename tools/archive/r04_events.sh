#!/bin/bash
# Cost of the per-step event records: events on every step vs every 10th vs none.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04events}"
mkdir -p "$OUT"
B=(--steps 100 --warmup 10 --no-cpu-baseline --no-variants --no-api --no-workloads)
run() {   # name every args...
  local name=$1 ev=$2; shift 2
  timeout -k 10 200 python bench.py "${B[@]}" --event-every $ev "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; [ $rc -le 1 ] || { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), r.get('kernel_ms'), round(d['value']/1e12,4))"
}
for r in 1 2; do
  for ev in 1 10 0; do
    run "full_e${ev}_$r" $ev
    run "strong8_e${ev}_$r" $ev --strong --nkeys 4096 --emulate-world 8
  done
done
