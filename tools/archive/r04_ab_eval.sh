#!/bin/bash
# configs[2] A/B: product library vs a build variant (DPF_LIB), interleaved.
#   tools/r04_ab_eval.sh <tag> <variant>...
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/$1"; shift
mkdir -p "$OUT"
lib() { if [ "$1" = base ]; then echo "$REPO/dpf-go_amd/lib/libdpf_hip.so"; else echo "$REPO/dpf-go_amd/lib/variants/libdpf_hip_$1.so"; fi; }
for r in 1 2; do
  for v in base "$@"; do
    DPF_LIB=$(lib $v) timeout -k 10 200 python bench.py --workload eval --steps 30 --warmup 5 --no-cpu-baseline --check \
        > "$OUT/eval_${v}_$r.log" 2>&1 || { echo "FAIL $v"; tail -5 "$OUT/eval_${v}_$r.log"; exit 1; }
    grep '^{' "$OUT/eval_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v r$r', round(d['ms_per_step'],4), 'kernel_ms', r['kernel_ms'], 'Gq', round(d['value']/1e9,3))"
  done
done
