#!/bin/bash
# r05: why batched Eval's walk runs at 0.85 of the LDS lookup rate where the
# tree kernel runs at 0.92: the same SQ counter passes over the configs[2]
# Eval step (k_eval_persist, and k_eval2 with DPF_EVAL_PERSIST=0) and the
# configs[1] EvalFull step (k_evalfull<7>).  One counter group per run.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/${1:-r05_pmc_eval}"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
C="--steps 5 --warmup 2 --spinup 0 --no-cpu-baseline --no-sweep --no-api --no-variants --no-workloads"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  for wl in eval evalfull; do
    timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/p${i}_$wl" -o p --output-format csv -- \
      python3 "$REPO/bench.py" --workload $wl $C > "$OUT/p${i}_$wl.log" 2>&1 || { echo "pass $i $wl failed"; tail -5 "$OUT/p${i}_$wl.log"; exit 1; }
  done
  DPF_EVAL_PERSIST=0 timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/p${i}_eval2" -o p --output-format csv -- \
      python3 "$REPO/bench.py" --workload eval $C > "$OUT/p${i}_eval2.log" 2>&1 || { echo "pass $i eval2 failed"; tail -5 "$OUT/p${i}_eval2.log"; exit 1; }
done
python3 "$REPO/tools/summarize_prof.py" "$OUT" > "$OUT/summary.json"
python3 - "$OUT/summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if k.startswith(("k_eval", "k_evalfull<7, true")):
        print(k, {c: round(x) for c, x in sorted(v.items())})
PY
