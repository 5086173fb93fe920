#!/bin/bash
# Rehearse the bench's multi-rank path on a 1-GPU box: 2 ranks (gloo for the
# barrier / max-reduce / PIR gather, both ranks on cuda:0) through torchrun,
# for every workload.  The driver's 8-GPU runs use RCCL (nccl) instead.
set -uo pipefail
mkdir -p gpurun_out/multirank
export DPF_BENCH_BACKEND=gloo
for w in evalfull eval split pir; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --workload $w --no-cpu-baseline \
      > gpurun_out/multirank/$w.log 2>&1
  rc=$?; echo "$w rc=$rc $(grep '^{' gpurun_out/multirank/$w.log | head -c 400)"
  [ $rc -eq 0 ] || exit $rc
done
