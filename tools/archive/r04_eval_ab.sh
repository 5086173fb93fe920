#!/bin/bash
# Batched Eval (configs[2]) A/B: k_eval2 one pair per thread (product) vs a
# resident-only grid (DPF_EVAL_STRIDE), with the next pair's inputs
# prefetched (DPF_EVAL_PREFETCH), with and without batched rounds.
# gpurun_out/evab/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/evab
mkdir -p $O
L=dpf-go_amd/lib/variants
run() {  # name lib
  DPF_LIB=$2 timeout -k 10 200 python bench.py --workload eval --steps 30 --warmup 5 --no-cpu-baseline > $O/$1.log 2>&1
}
for r in 1 2; do
  run base_$r dpf-go_amd/lib/libdpf_hip.so || exit $?
  for v in evs evsp evspnb; do run ${v}_$r $L/libdpf_hip_$v.so || exit $?; done
done
