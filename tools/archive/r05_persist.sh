#!/bin/bash
# r05: persistent batched Eval (k_eval_persist: one workgroup per CU, table
# filled once, next pair's points and frontier nodes staged by LDS-DMA) vs
# k_eval2 at configs[2]; Eval parity tests with the persistent kernel first.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_persist}"; mkdir -p "$OUT"
export TMPDIR=/tmp
DPF_EVAL_PERSIST=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
   tests/test_gpu_eval_configs.py tests/test_gpu_parity.py -k "eval or config2" > "$OUT/tests.log" 2>&1 \
   || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
B="--workload eval --steps 40 --warmup 5 --no-cpu-baseline"
for round in 1 2 3; do
  for u in 1 0; do
    DPF_EVAL_PERSIST=$u timeout -k 10 120 python3 bench.py $B > "$OUT/eval_p${u}_$round.log" 2>&1 || { echo "bench p=$u failed"; tail -5 "$OUT/eval_p${u}_$round.log"; exit 1; }
    grep '^{' "$OUT/eval_p${u}_$round.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('persist=$u round $round', round(d['ms_per_step'],4), 'ms', round(d['value']/1e9,3), 'G q/s kernel', d['roofline']['kernel_ms'])" | tee -a "$OUT/ab.txt"
  done
done
( cd /tmp && DPF_EVAL_PERSIST=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" $B > "$REPO/$OUT/kt.log" 2>&1 ) || { echo "kt failed"; exit 1; }
rm -f "$OUT"/kt/*kernel_trace.csv
python3 - "$OUT/kt/kt_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"].split("(")[0][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
# PIR tree of batch i+1 beside the fold of batch i on a second stream, at the
# N = 8 / 4 rank shapes (prefix 3 / 2) and on one GPU.
for pb in 3 2 0; do
  PB=$pb timeout -k 10 120 python3 tools/pir_overlap.py 300 > "$OUT/overlap_pb$pb.log" 2>&1 || { echo "overlap pb=$pb failed"; tail -5 "$OUT/overlap_pb$pb.log"; exit 1; }
  echo "pb=$pb $(tail -1 "$OUT/overlap_pb$pb.log")" | tee -a "$OUT/ab.txt"
done
# The fold's ablations again with nontemporal DB loads (the product at 2^24).
export FOLD_MODE=mfma
for r in 1 2 3; do
  for b in fold_bench bin/fold_bench_ablate1 bin/fold_bench_ablate2; do
    timeout -k 10 60 tools/$b 64 32 24 > "$OUT/ab.json" 2>&1
    rc=$?   # the ablation builds compute wrong answers on purpose (exit 1, "ok": false)
    if [ $rc -ne 0 ] && ! grep -q '"fold_us"' "$OUT/ab.json"; then echo "$b failed rc=$rc"; cat "$OUT/ab.json"; exit 1; fi
    python3 -c "import json; d=json.load(open('$OUT/ab.json')); print('$r $(basename $b) 64 32 24', d['fold_us'], 'us', d['GBs'], 'GB/s')" | tee -a "$OUT/ablate_nt.txt"
  done
done
