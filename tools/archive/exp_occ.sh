#!/bin/bash
# A/B of tree-kernel build variants (interleaved runs, same process layout):
#   base  : 512-thread WGs, 4 waves/SIMD, PRG MMOs interleaved
#   occ5  : 640-thread WGs, 5 waves/SIMD (VGPR spills)
#   ilp1  : PRG MMOs serialized
set -uo pipefail
mkdir -p gpurun_out/exp3
for r in 1 2; do
  for v in base ilp2 ilp1; do
    if [ $v = base ]; then unset DPF_LIB; else export DPF_LIB=$PWD/dpf-go_amd/lib/variants/libdpf_hip_$v.so; fi
    timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --check > gpurun_out/exp3/full_${v}_$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.e+]*' gpurun_out/exp3/full_${v}_$r.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/exp3/full_${v}_$r.log)"
  done
done
