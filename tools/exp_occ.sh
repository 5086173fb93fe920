#!/bin/bash
# A/B: tree kernel at 4 waves/SIMD (512-thread WGs) vs 5 waves/SIMD (640, spills), interleaved runs.
set -uo pipefail
mkdir -p gpurun_out/exp3
for r in 1 2; do
  for v in base occ5; do
    if [ $v = occ5 ]; then export DPF_LIB=$PWD/dpf-go_amd/lib/variants/libdpf_hip_occ5.so; else unset DPF_LIB; fi
    timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --check > gpurun_out/exp3/full_${v}_$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.e+]*' gpurun_out/exp3/full_${v}_$r.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/exp3/full_${v}_$r.log)"
  done
done
