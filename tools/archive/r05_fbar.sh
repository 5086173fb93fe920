#!/bin/bash
# r05: the folds' LDS-only barrier (DPF_FOLD_RAW_BARRIER, lds_barrier) vs
# __syncthreads(), with one or two staged blocks in flight (DPF_FOLD_PD), at
# B = 64 and 256 over 2^24 records (and 2^21: the N = 8 rank), plus the
# loads-only ablation under the new barrier.  tools/fold_bench builds in
# tools/ and tools/bin.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fbar}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for r in 1 2 3; do
  for b in fold_bench bin/fold_bench_pd2 bin/fold_bench_sync bin/fold_bench_sync_pd2 bin/fold_bench_ablate1 bin/fold_bench_ablate1_pd2; do
    for cfg in "64 32 24" "64 32 21" "256 32 24"; do
      timeout -k 10 60 tools/$b $cfg > "$OUT/fb.json" 2>&1
      rc=$?
      if [ $rc -ne 0 ] && ! grep -q '"fold_us"' "$OUT/fb.json"; then echo "$b failed rc=$rc"; cat "$OUT/fb.json"; exit 1; fi
      python3 -c "import json; d=json.load(open('$OUT/fb.json')); print('$r $(basename $b) $cfg', d['fold_us'], 'us', d['GBs'], 'GB/s ok', d['ok'])" | tee -a "$OUT/fbar.txt"
    done
  done
done
