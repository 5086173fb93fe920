#!/bin/bash
# Issue-priority thresholds for the 32-group threads of configs[1] (D = 7):
# product 3/4, 7/8, 15/16 vs 1/2, 3/4, 7/8 (big2) vs 7/8, 15/16, 31/32
# (big5); configs[1] line, 3 interleaved rounds.  gpurun_out/prio3/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/prio3
mkdir -p $O
L=dpf-go_amd/lib/variants
for r in 1 2 3; do
  for v in s3:dpf-go_amd/lib/libdpf_hip.so big2:$L/libdpf_hip_big2.so big5:$L/libdpf_hip_big5.so; do
    n=${v%%:*}; lib=${v#*:}
    DPF_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-variants --no-api --no-workloads > $O/c1_${n}_$r.log 2>&1 || exit $?
  done
done
