#!/bin/bash
# PIR step with DPF_FOLD_SKEW 50 (even split) vs 62, 3 interleaved rounds.
set -o pipefail
B="--workload pir --steps 40 --warmup 5 --no-cpu-baseline --no-variants --no-api --no-sweep"
for r in 1 2 3; do
  for k in 50 62; do
    DPF_FOLD_SKEW=$k timeout -k 10 120 python bench.py $B > gpurun_out/pir_skew_${k}_$r.log 2>&1 || exit 1
    grep '^{' gpurun_out/pir_skew_${k}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('skew $k r$r', round(d['ms_per_step'],4), d['roofline']['kernel_ms'])"
  done
done
