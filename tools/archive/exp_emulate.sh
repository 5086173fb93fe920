#!/bin/bash
# Rank 0's share of the strong-scaling workloads (configs[3] split, configs[4]
# PIR) timed on one GPU for N = 1, 2, 4, 8 (--emulate-world): the per-rank
# time the driver's N-GPU runs will see, before any collective.
set -o pipefail
out=gpurun_out/emulate; mkdir -p $out
for w in split pir; do
  for n in 1 2 4 8; do
    timeout -k 10 120 python bench.py --workload $w --emulate-world $n --steps 30 --warmup 5 --no-cpu-baseline \
        --no-variants --no-api --no-sweep > $out/${w}_$n.log 2>&1 || { tail -5 $out/${w}_$n.log; exit 1; }
    grep '^{' $out/${w}_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w N=$n', round(d['ms_per_step'],4), 'kernels', d['roofline']['kernel_ms'], 'value', d['value'])"
  done
done
