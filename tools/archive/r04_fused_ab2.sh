#!/bin/bash
# k_pir_fused producer rate with 16 producer waves (4 per SIMD), no folders
# (DPF_FZ_PRODONLY; answers not meaningful), plain and batched AES rounds,
# against the 12-producer no-fold variant.  gpurun_out/fz/ab2/.
# The DPF_FZ_PRODONLY switch (kFzProd = 16, kFzFold = 0, one ring slot, no
# flow control) was a measurement-only edit of the v3 kernel and was not
# committed; the results are in profiles/r04/fused/ab2_*.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/fz/${1:-ab2}
mkdir -p $O
L=dpf-go_amd/lib/variants
run() {  # name lib
  DPF_LIB=$2 DPF_PIR_KERNEL=fused timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep > $O/$1.log 2>&1
}
for r in 1 2; do
  for v in fzprod16 fzprod16b fznofold fzbatchnofold; do run ${v}_$r $L/libdpf_hip_$v.so || exit $?; done
done
