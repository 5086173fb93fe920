#!/bin/bash
# Issue-priority schemes (DPF_PRIO_STEPS 3 = product: 3/4, 7/8, 15/16 of a
# thread's 4-leaf groups; 2: 1/2, 3/4, 7/8; 1: 1/4, 1/2, 3/4) at the PIR
# tree's shape (8 groups per thread) and at configs[1]: PIR line (tree timed
# apart) and per-wave end spread.  gpurun_out/prio/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/prio
mkdir -p $O
L=dpf-go_amd/lib/variants
for r in 1 2; do
  DPF_LIB=dpf-go_amd/lib/libdpf_hip.so timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep > $O/pir_s3_$r.log 2>&1 || exit $?
  for s in 1 2; do
    DPF_LIB=$L/libdpf_hip_prio$s.so timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep > $O/pir_s${s}_$r.log 2>&1 || exit $?
  done
done
for r in 1 2; do
  timeout -k 10 120 tools/bin/wave_times 64 24 | sed 's/^{/{"scheme": 3, /' >> $O/wt.jsonl || exit $?
  for s in 1 2; do timeout -k 10 120 tools/bin/wave_times_s$s 64 24 | sed "s/^{/{\"scheme\": $s, /" >> $O/wt.jsonl || exit $?; done
done
