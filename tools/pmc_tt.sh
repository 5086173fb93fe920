#!/bin/bash
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/pmc_tt"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- "$REPO/tools/bin/tt_bench" > "$OUT/p$i.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p${i}b" -o p${i}b --output-format csv -- python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-api --no-variants > "$OUT/p${i}b.log" 2>&1 || exit 1
done
python3 "$REPO/tools/summarize_prof.py" "$OUT" > "$OUT/summary.json"
python3 - "$OUT/summary.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    if 'tt' in k or 'evalfull' in k:
        print(k, {c: round(x) for c,x in v.items()})
PY
