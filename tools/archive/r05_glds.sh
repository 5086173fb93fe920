#!/bin/bash
# r05: the LDS-DMA fold (k_fold_glds, DPF_FOLD_GLDS=1..4) vs k_fold_mfma at
# B = 64: fold parity tests under each mode, tools/fold_bench interleaved,
# then the PIR step; plus the quad walk's fan-out (variant fan7) A/B.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_glds}"; mkdir -p "$OUT"
export FOLD_MODE=mfma
for g in 1 3; do
  DPF_FOLD_GLDS=$g timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
     tests/test_gpu_fold.py tests/test_gpu_per_rank.py -k "sliced or config4 or fold" > "$OUT/tests_g$g.log" 2>&1 \
     || { tail -30 "$OUT/tests_g$g.log"; exit 1; }
  echo "glds=$g: $(tail -1 $OUT/tests_g$g.log)"
done
for r in 1 2 3; do
  for g in 0 1 2 3 4; do
    for lg in 24 21; do
      DPF_FOLD_GLDS=$g timeout -k 10 60 tools/fold_bench 64 32 $lg > "$OUT/fb_g${g}_${lg}_$r.json" 2>&1 || { echo "fold_bench g=$g failed"; cat "$OUT/fb_g${g}_${lg}_$r.json"; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/fb_g${g}_${lg}_$r.json')); print('$r glds=$g logN=$lg', d['fold_us'], 'us', d['GBs'], 'GB/s ok', d['ok'])"
    done
  done
done
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
for r in 1 2; do
  for g in 0 1 3; do
    for w in 1 8; do
      DPF_FOLD_GLDS=$g timeout -k 10 120 python3 bench.py $C --workload pir --emulate-world $w > "$OUT/pir_g${g}_w${w}_$r.log" 2>&1 || { echo "pir failed"; exit 1; }
      grep '^{' "$OUT/pir_g${g}_w${w}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$r glds=$g W=$w step', round(d['ms_per_step'],4), 'fold', k['fold']['kernel_ms'])"
    done
  done
done
for r in 1 2; do
  for s in "--workload pir --emulate-world 8" "--workload split --emulate-world 8" "--strong --nkeys 4096 --emulate-world 8"; do
    for L in dpf-go_amd/lib/libdpf_hip.so dpf-go_amd/lib/variants/libdpf_hip_fan7.so; do
      DPF_LIB="$REPO/$L" timeout -k 10 120 python3 bench.py $C $s > "$OUT/fan.log" 2>&1 || { echo "FAIL fan"; exit 1; }
      grep '^{' "$OUT/fan.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r', '$s'.split()[1], '$(basename $L .so)', round(d['ms_per_step'],4), 'ms kernel', d['roofline'].get('kernel_ms'))"
    done
  done
done
bash tools/archive/r05_depth.sh r05_depth
bash tools/archive/r05_small.sh r05_small
