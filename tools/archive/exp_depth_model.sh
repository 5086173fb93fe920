#!/bin/bash
# The coop-aware depth model's two changed choices (PIR rank at N=4: D 4 -> 3,
# N=8: D 3 -> 2) against the forced old ones, 2 interleaved rounds.
set -o pipefail
B="--workload pir --steps 30 --warmup 5 --no-cpu-baseline --no-variants --no-api --no-sweep"
for r in 1 2; do
  for cfg in "4 auto" "4 4" "8 auto" "8 3"; do
    set -- $cfg
    if [ $2 = auto ]; then unset DPF_SUBTREE_DEPTH; else export DPF_SUBTREE_DEPTH=$2; fi
    timeout -k 10 120 python bench.py $B --emulate-world $1 > gpurun_out/dm_$1_$2_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/dm_$1_$2_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$1 D=$2 r$r', round(d['ms_per_step'],4), d['roofline']['kernel_ms'])"
  done
  unset DPF_SUBTREE_DEPTH
done
