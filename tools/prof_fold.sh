#!/bin/bash
# PMC passes over the fold microbenchmark binaries (tools/bin/fold_bench_*).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/${1:-gpurun_out/pf}"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
for b in r01 new; do
  mkdir -p "$OUT/$b"
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp -d "$OUT/$b/p$i" -o p$i --output-format csv -- "$REPO/tools/bin/fold_bench_$b" > "$OUT/$b/p$i.log" 2>&1 || { echo "fail $b $i"; exit 1; }
  done
  python3 "$REPO/tools/summarize_prof.py" "$OUT/$b" > "$OUT/$b/summary.json"
done
echo ok
