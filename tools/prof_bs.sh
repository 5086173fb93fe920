#!/bin/bash
# Kernel trace + PMC passes of the configs[1] bench on one AES back end.
# Usage: tools/prof_bs.sh <out_dir> <ttable|bitsliced>
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/$1"; IMPL="$2"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B=(python3 "$REPO/bench.py" --aes "$IMPL" --no-variants --no-cpu-baseline --steps 10 --warmup 3)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${B[@]}" > "$OUT/kt.log" 2>&1 || exit 1
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
           "WRITE_SIZE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- "${B[@]}" > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python3 "$REPO/tools/summarize_prof.py" "$OUT" > "$OUT/summary.json"
echo "done $OUT"
