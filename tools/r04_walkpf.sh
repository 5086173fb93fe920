#!/bin/bash
# Walk prefetch (product) vs DPF_WALK_PREFETCH=0 (variant lib), interleaved:
# configs[1] headline, strong per-rank shapes, split and PIR lines.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04walkpf}"
mkdir -p "$OUT"
B=(--steps 50 --warmup 10 --no-cpu-baseline --no-variants --no-api --no-workloads)
lib() { if [ "$1" = base ]; then echo "$REPO/dpf-go_amd/lib/libdpf_hip.so"; else echo "$REPO/dpf-go_amd/lib/variants/libdpf_hip_$1.so"; fi; }
run() {   # name variant args...
  local name=$1 v=$2; shift 2
  DPF_LIB=$(lib $v) timeout -k 10 200 python bench.py "${B[@]}" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; [ $rc -le 1 ] || { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), r['kernel_ms'], round(d['value']/1e12,4))"
}
for r in 1 2; do
  for v in base nowalkpf; do
    run "full_${v}_$r" $v --check
    for w in 4 8; do run "strong${w}_${v}_$r" $v --strong --nkeys 4096 --emulate-world $w; done
    run "split_${v}_$r" $v --workload split --check
    run "pir_${v}_$r" $v --workload pir --no-sweep --check
  done
done
