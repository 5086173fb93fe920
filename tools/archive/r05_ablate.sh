#!/bin/bash
# r05: what the matrix-core fold's time is made of (k_fold_mfma<2,2,2,1>,
# B = 64, 2^24 records): the product kernel, a build that only loads and
# stages its operands (DPF_FOLD_ABLATE=1: no FP4 expansion, no MFMA), and a
# build that computes without reading HBM (DPF_FOLD_ABLATE=2); then the quad
# walk's fan-out (variant fan7), the depth sweep and the small-call
# thresholds.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_ablate}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for r in 1 2 3; do
  for b in fold_bench bin/fold_bench_ablate1 bin/fold_bench_ablate2; do
    for lg in 24 21; do
      timeout -k 10 60 tools/$b 64 32 $lg > "$OUT/ab.json" 2>&1
      rc=$?   # the ablation builds compute wrong answers on purpose: fold_bench exits 1 ("ok": false)
      if [ $rc -ne 0 ] && ! grep -q '"fold_us"' "$OUT/ab.json"; then echo "$b failed rc=$rc"; cat "$OUT/ab.json"; exit 1; fi
      python3 -c "import json; d=json.load(open('$OUT/ab.json')); print('$r $(basename $b) logN=$lg', d['fold_us'], 'us', d['GBs'], 'GB/s')" | tee -a "$OUT/ablate.txt"
    done
  done
done
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
for r in 1 2; do
  for s in "--workload pir --emulate-world 8" "--workload split --emulate-world 8" "--strong --nkeys 4096 --emulate-world 8"; do
    for L in dpf-go_amd/lib/libdpf_hip.so dpf-go_amd/lib/variants/libdpf_hip_fan7.so; do
      DPF_LIB="$REPO/$L" timeout -k 10 120 python3 bench.py $C $s > "$OUT/fan.log" 2>&1 || { echo "FAIL fan"; tail -3 "$OUT/fan.log"; exit 1; }
      grep '^{' "$OUT/fan.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$s'.split()[1], '$(basename $L .so)', round(d['ms_per_step'],4), 'ms kernel', d['roofline'].get('kernel_ms'))" | tee -a "$OUT/fan.txt"
    done
  done
done
bash tools/archive/r05_depth.sh r05_depth
bash tools/archive/r05_small.sh r05_small
