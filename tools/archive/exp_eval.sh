#!/bin/bash
# A/B of tree-kernel build variants on the Eval workload (configs[2]),
# interleaved over 3 rounds, plus a kernel trace per variant.
#   tools/exp_eval.sh <out_tag> <variant>...   ("base" = product build)
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/$1"; shift
mkdir -p "$OUT"
B=(--workload eval --steps 30 --warmup 5 --spinup 0.5 --no-cpu-baseline --no-variants --no-api --aes ttable)
lib() { if [ "$1" = base ]; then echo "$REPO/dpf-go_amd/lib/libdpf_hip.so"; else echo "$REPO/tools/bin/libdpf_hip_$1.so"; fi; }
for r in 1 2 3; do
  for v in "$@"; do
    DPF_LIB=$(lib $v) timeout -k 10 200 python bench.py "${B[@]}" --check > "$OUT/${v}_$r.log" 2>&1 || { echo "FAIL $v"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
    grep '^{' "$OUT/${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v r$r', round(d['ms_per_step'],4), d['value'])"
  done
done
export TMPDIR=/tmp
for v in "$@"; do
  ( cd /tmp && DPF_LIB=$(lib $v) timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/t_$v" -o t --output-format csv -- \
      python3 "$REPO/bench.py" --workload eval --steps 10 --warmup 2 --no-cpu-baseline --no-variants --no-api --aes ttable > "$REPO/$OUT/t_$v.log" 2>&1 ) || { echo "trace FAIL $v"; exit 1; }
  f=$(find "$REPO/$OUT/t_$v" -name '*kernel_stats.csv' | head -1)
  echo "$v"; grep -E 'k_eval|k_evalfull' "$f" | cut -d, -f1-6
done
