#!/bin/bash
# Shared (workgroup) walk vs per-thread walk (variant "nocoop"): parity tests,
# then PIR / split / default bench lines for both builds, interleaved.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-coop}"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for r in 1 2; do
  for v in base nocoop; do
    L="$REPO/dpf-go_amd/lib/libdpf_hip.so"; [ $v = nocoop ] && L="$REPO/dpf-go_amd/lib/variants/libdpf_hip_nocoop.so"
    for w in pir split evalfull eval; do
      DPF_LIB=$L timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline --no-api --no-variants --check > "$OUT/${w}_${v}_$r.log" 2>&1 || { echo "FAIL $w $v"; tail -5 "$OUT/${w}_${v}_$r.log"; exit 1; }
      grep '^{' "$OUT/${w}_${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w $v r$r', round(d['ms_per_step'],4), d['roofline']['kernel_ms'])"
    done
  done
done
