#!/bin/bash
# r05: k_xor_parts (64 atomics per answer word) vs the two-stage
# k_xor_parts2 (DPF_XOR_PARTS=2: LDS-combined, one atomic per word per block),
# and nontemporal operand loads in k_fold_mfma (DPF_FOLD_NT=1 DB, 2 DB + sel),
# on tools/fold_bench at B = 64 over 2^24 and 2^21 records (the N = 8 rank)
# and B = 256; then a kernel trace of both partial-XOR forms.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_xp}"; mkdir -p "$OUT"
export FOLD_MODE=mfma TMPDIR=/tmp
for r in 1 2 3; do
  for b in fold_bench bin/fold_bench_xp2 bin/fold_bench_nt1 bin/fold_bench_nt2; do
    for cfg in "64 32 24" "64 32 21" "256 32 24"; do
      timeout -k 10 60 tools/$b $cfg > "$OUT/fb.json" 2>&1 || { echo "$b $cfg failed"; cat "$OUT/fb.json"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r $(basename $b) $cfg', d['fold_us'], 'us', d['GBs'], 'GB/s ok', d['ok'])" | tee -a "$OUT/xp.txt"
    done
  done
done
for b in fold_bench bin/fold_bench_xp2; do
  n=$(basename $b)
  ( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_$n" -o kt --output-format csv -- \
      "$REPO/tools/$b" 64 32 21 > "$REPO/$OUT/kt_$n.log" 2>&1 ) || { echo "kt $n failed"; exit 1; }
  rm -f "$OUT"/kt_$n/*kernel_trace.csv
  grep -h "xor_parts\|fold_mfma" "$OUT"/kt_$n/*kernel_stats.csv | cut -d, -f1-4 | sed 's/(.*)"/"/' | tee -a "$OUT/xp.txt"
done
