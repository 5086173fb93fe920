#!/bin/bash
# r05: one matrix-core fold workgroup per CU (DPF_FOLD_PER_CU=1: a third of
# the partials for k_xor_parts) against 2 per CU (the policy before the
# change; PCS picks the pair, default "0 1") at the per-rank PIR shapes,
# interleaved.  Arg 2 = tests: the fold and per-rank GPU tests first.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fpercu1}"; mkdir -p "$OUT"
if [ "${2:-}" = tests ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fold.py tests/test_gpu_per_rank.py tests/test_gpu_pir_fused.py -m gpu -x -q \
      --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads --workload pir"
for r in 1 2 3; do
  for W in ${WS:-8 4}; do
    for pc in ${PCS:-0 1}; do
      DPF_FOLD_PER_CU=$pc timeout -k 10 120 python3 bench.py $C --emulate-world $W > "$OUT/pir.log" 2>&1 || { echo "FAIL pir"; tail -3 "$OUT/pir.log"; exit 1; }
      grep '^{' "$OUT/pir.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$r W=$W per_cu=$pc', round(d['ms_per_step'],4), 'fold', k['fold']['kernel_ms'])" | tee -a "$OUT/pir.txt"
    done
  done
done
