#!/bin/bash
# Raw-key tree path (no unpack launch) vs DPF_RAW_KEYS=0, interleaved: the
# default headline, configs[1] strong per-rank shapes, split and PIR lines.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04raw}"
mkdir -p "$OUT"
B=(--steps 50 --warmup 10 --no-cpu-baseline --no-variants --no-api --no-workloads)
run() {   # name raw args...
  local name=$1 raw=$2; shift 2
  DPF_RAW_KEYS=$raw timeout -k 10 200 python bench.py "${B[@]}" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; [ $rc -le 1 ] || { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), r['kernel_ms'], round(d['value']/1e12,4))"
}
for r in 1 2; do
  for raw in 1 0; do
    run "full_raw${raw}_$r" $raw --check
    for w in 2 4 8; do run "strong${w}_raw${raw}_$r" $raw --strong --nkeys 4096 --emulate-world $w; done
    run "split_raw${raw}_$r" $raw --workload split --check
    run "pir_raw${raw}_$r" $raw --workload pir --no-sweep --check
  done
done
