#!/bin/bash
# Lane-pair whole-line leaf stores (product) vs r02 half-line stores (variant
# "half"): parity tests, default A/B with WRITE_SIZE, PIR and split lines.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-pair}"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -20 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
bash tools/exp_variants.sh "${1:-pair}/ab" base half || exit 1
for v in base half; do
  L="$REPO/dpf-go_amd/lib/libdpf_hip.so"; [ $v = half ] && L="$REPO/dpf-go_amd/lib/variants/libdpf_hip_half.so"
  for w in pir split; do
    DPF_LIB=$L timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > "$OUT/${w}_$v.log" 2>&1 || { echo "FAIL $w $v"; exit 1; }
    grep '^{' "$OUT/${w}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w $v', round(d['ms_per_step'],4), d['roofline']['kernel_ms'])"
  done
done
