#!/bin/bash
# A/B of build variants (lib/variants/libdpf_hip_<v>.so; "base" = the product
# library), interleaved runs, parity first.
# Usage: tools/exp_ab.sh "<workloads>" <variant>...   e.g. tools/exp_ab.sh "evalfull pir" base lastl1
set -uo pipefail
WL="$1"; shift
OUT=gpurun_out/ab
mkdir -p $OUT
for v in "$@"; do
  [ $v = base ] && continue
  DPF_LIB=$PWD/dpf-go_amd/lib/variants/libdpf_hip_$v.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py \
      tests/test_gpu_pir.py -m gpu -x -q > $OUT/parity_$v.log 2>&1 || { echo "parity FAILED for $v"; tail -20 $OUT/parity_$v.log; exit 1; }
  echo "parity ok: $v"
done
for r in 1 2; do
  for w in $WL; do
    for v in "$@"; do
      if [ $v = base ]; then unset DPF_LIB; else export DPF_LIB=$PWD/dpf-go_amd/lib/variants/libdpf_hip_$v.so; fi
      timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 10 --no-cpu-baseline > $OUT/${w}_${v}_$r.log 2>&1 || exit 1
      echo "$w $v r$r $(grep -o '"value": [0-9.e+]*' $OUT/${w}_${v}_$r.log) $(grep -o '"kernel_ms": [0-9.]*' $OUT/${w}_${v}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' $OUT/${w}_${v}_$r.log)"
    done
  done
done
