#!/bin/bash
# MFMA (FP4) fold vs the LDS fold at configs[4] shape: fold_bench over
# B = 1..256 in both modes, the sliced-fold GPU tests, and a rocprofv3 kernel
# trace + PMC passes (FETCH, MFMA busy, LDS busy) of both at B = 64 and 256.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04fold}"
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py -v --timeout 120 --timeout-method thread -k sliced \
    > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/tests.log"
[ $rc -le 1 ] || exit $rc
for b in 1 4 8 16 32 64 128 256 512; do
  for m in lds mfma; do
    FOLD_MODE=$m timeout -k 10 120 tools/fold_bench $b 32 24 >> "$OUT/fold_bench.jsonl" 2>> "$OUT/fold_bench.err"
    rc=$?; [ $rc -le 1 ] || { echo "fold_bench $m $b rc=$rc"; exit $rc; }
  done
done
cat "$OUT/fold_bench.jsonl"
export TMPDIR=/tmp
for b in 64 256; do
  for m in lds mfma; do
    ( cd /tmp && FOLD_MODE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_${m}_$b" -o kt \
        --output-format csv -- "$REPO/tools/fold_bench" $b 32 24 > /dev/null 2>&1 ); echo "kt $m $b rc=$?"
    i=0
    for grp in "FETCH_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
               "SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE"; do
      i=$((i+1))
      ( cd /tmp && FOLD_MODE=$m timeout -s KILL 90 rocprofv3 --pmc $grp -d "$REPO/$OUT/pmc_${m}_${b}_$i" -o p \
          --output-format csv -- "$REPO/tools/fold_bench" $b 32 24 > /dev/null 2>&1 ); echo "pmc $m $b $i rc=$?"
    done
  done
done
echo done
