#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains) over
# one bench workload.  Usage: tools/counters.sh <out_dir> <workload> [bench args...]
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/$1"; WL="$2"; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH=(python3 "$REPO/bench.py" --workload "$WL" --steps 5 --warmup 2 --no-cpu-baseline --no-sweep --no-api --no-variants --no-workloads "$@")
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VALU SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU" \
           "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- "${BENCH[@]}" > "$OUT/p$i.log" 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${BENCH[@]}" \
    > "$OUT/kt.log" 2>&1
python3 "$REPO/tools/summarize_prof.py" "$OUT" > "$OUT/summary.json"
cat "$OUT/summary.json"
