#!/bin/bash
# Issue priority for subtrees of <= 2^5 leaf blocks: product (1/2, 3/4, 7/8)
# vs the configs[1] scheme everywhere (variant prio33: 3/4, 7/8, 15/16), on
# the shapes that use them: the PIR tree, configs[1] strong scaling at 4 and
# 8 ranks, configs[3] per-rank at 8; interleaved.  gpurun_out/prio2/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/prio2
mkdir -p $O
A=dpf-go_amd/lib/libdpf_hip.so
B=dpf-go_amd/lib/variants/libdpf_hip_prio33.so
for r in 1 2; do
  for v in new:$A old:$B; do
    n=${v%%:*}; lib=${v#*:}
    DPF_LIB=$lib timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep > $O/pir_${n}_$r.log 2>&1 || exit $?
    for w in 4 8; do
      DPF_LIB=$lib timeout -k 10 200 python bench.py --strong --nkeys 4096 --emulate-world $w --steps 200 --warmup 20 --no-cpu-baseline --no-variants --no-api --no-workloads > $O/strong${w}_${n}_$r.log 2>&1 || exit $?
    done
    DPF_LIB=$lib timeout -k 10 200 python bench.py --workload split --emulate-world 8 --steps 100 --warmup 10 --no-cpu-baseline --no-api > $O/split8_${n}_$r.log 2>&1 || exit $?
  done
done
