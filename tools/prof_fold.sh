#!/bin/bash
# PMC passes over fold microbenchmark runs.  Usage:
#   tools/prof_fold.sh <out_dir> <name>=<binary>:<args> ...
# e.g. new64=tools/fold_bench:"64 32 24"  r02=tools/bin/fold_bench_r02:"64 32 24"
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/$1"; shift; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
for spec in "$@"; do
  name="${spec%%=*}"; rest="${spec#*=}"; bin="${rest%%:*}"; args="${rest#*:}"
  mkdir -p "$OUT/$name"
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp -d "$OUT/$name/p$i" -o p$i --output-format csv -- "$REPO/$bin" $args \
      > "$OUT/$name/p$i.log" 2>&1 || { echo "fail $name $i"; tail -5 "$OUT/$name/p$i.log"; exit 1; }
  done
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d "$OUT/$name/kt" -o kt --output-format csv -- "$REPO/$bin" $args \
    > "$OUT/$name/kt.log" 2>&1 || { echo "fail $name kt"; exit 1; }
  python3 "$REPO/tools/summarize_prof.py" "$OUT/$name" > "$OUT/$name/summary.json"
done
echo ok
