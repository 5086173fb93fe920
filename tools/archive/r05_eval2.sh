#!/bin/bash
# r05: k_eval2 with wave-uniform keys (CWs in SGPRs) vs per-lane keys
# (DPF_EVAL_UNIFORM=0) at configs[2], Eval parity tests on the product and
# the experimental build, then the fold's PMC passes (tools/archive/r05_pmc_fold.sh).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_eval2}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_eval_configs.py \
   tests/test_gpu_parity.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
DPF_LIB=dpf-go_amd/lib/variants/libdpf_hip_exp.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 \
   --timeout-method thread -m gpu tests/test_gpu_eval_configs.py tests/test_gpu_pir_fused.py > "$OUT/tests_exp.log" 2>&1 \
   || { tail -30 "$OUT/tests_exp.log"; exit 1; }
tail -1 "$OUT/tests_exp.log"
B="--workload eval --steps 40 --warmup 5 --no-cpu-baseline"
for round in 1 2 3; do
  for u in 1 0; do
    DPF_EVAL_UNIFORM=$u timeout -k 10 120 python3 bench.py $B > "$OUT/eval_u${u}_$round.log" 2>&1 || { echo "bench u=$u failed"; tail -5 "$OUT/eval_u${u}_$round.log"; exit 1; }
    grep '^{' "$OUT/eval_u${u}_$round.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('uniform=$u round $round', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G q/s kernel', d['roofline']['kernel_ms'])"
  done
done
bash tools/archive/r05_pmc_fold.sh r05_pmc_fold64 > "$OUT/pmc64.txt" 2>&1; tail -3 "$OUT/pmc64.txt"
