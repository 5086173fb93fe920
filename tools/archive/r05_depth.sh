#!/bin/bash
# r05: per-thread subtree depth D (DPF_SUBTREE_DEPTH) at the small per-rank
# shapes with the quad-form shared walk, against the depth model's choice.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_depth}"; mkdir -p "$OUT"
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
declare -A SH
SH[pir8]="--workload pir --emulate-world 8"
SH[pir4]="--workload pir --emulate-world 4"
SH[split8]="--workload split --emulate-world 8"
SH[strong8]="--strong --nkeys 4096 --emulate-world 8"
for s in pir8 pir4 split8 strong8; do
  for d in auto 1 2 3 4 5 6; do
    if [ $d = auto ]; then unset DPF_SUBTREE_DEPTH; else export DPF_SUBTREE_DEPTH=$d; fi
    timeout -k 10 120 python3 bench.py $C ${SH[$s]} > "$OUT/${s}_d$d.log" 2>&1 || { echo "FAIL $s $d"; tail -3 "$OUT/${s}_d$d.log"; exit 1; }
    grep '^{' "$OUT/${s}_d$d.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$s D=$d', round(d['ms_per_step'],4), 'ms kernel', d['roofline'].get('kernel_ms'))"
  done
  unset DPF_SUBTREE_DEPTH
done
