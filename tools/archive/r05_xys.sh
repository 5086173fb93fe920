#!/bin/bash
# r05: k_xor_parts part slices per answer word (DPF_XOR_PARTS_YS: atomics per
# word) at the PIR rank (N = 8) and on one GPU, interleaved, with --check on
# the first round.  YS=0 runs the library's default.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_xys}"; mkdir -p "$OUT"
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads --workload pir"
for r in 1 2 3; do
  for W in ${WS:-8 1}; do
    for ys in ${YS:-64 16 8}; do
      if [ $ys = 0 ]; then unset DPF_XOR_PARTS_YS; else export DPF_XOR_PARTS_YS=$ys; fi
      timeout -k 10 120 python3 bench.py $C --emulate-world $W $( [ $r = 1 ] && [ $W = 1 ] && echo --check ) > "$OUT/pir.log" 2>&1 || { echo "FAIL ys=$ys W=$W"; tail -3 "$OUT/pir.log"; exit 1; }
      grep '^{' "$OUT/pir.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$r W=$W ys=$ys', round(d['ms_per_step'],4), 'fold+xor', k['fold']['kernel_ms'])" | tee -a "$OUT/pir.txt"
    done
  done
done
