#!/bin/bash
# k_pir_fused A/B over build variants (tools/build_variant.sh): producer AES
# batching, no fold (producer rate alone), no L2 touch.  gpurun_out/fz/ab/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/fz/${1:-ab}
mkdir -p $O
L=dpf-go_amd/lib/variants
run() {  # name lib
  DPF_LIB=$2 DPF_PIR_KERNEL=fused timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep > $O/$1.log 2>&1
}
DPF_PIR_KERNEL=split timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep > $O/split.log 2>&1 || exit $?
for r in 1 2; do
  run base_$r dpf-go_amd/lib/libdpf_hip.so || exit $?
  for v in fzbatch fznofold fznotouch fzbatchnofold; do run ${v}_$r $L/libdpf_hip_$v.so || exit $?; done
done
