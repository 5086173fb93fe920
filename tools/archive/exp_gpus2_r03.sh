#!/bin/bash
# 2-rank rehearsal on a 1-GPU box (ranks folded onto cuda:0 over gloo, the
# line marks folded_ranks): every workload's N>1 path runs end to end.
set -o pipefail
out=gpurun_out/gpus2_r03; mkdir -p $out
for w in evalfull eval split pir; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --workload $w --check --no-sweep --no-api \
      --no-variants > $out/$w.log 2>&1 || { echo "FAIL $w"; tail -20 $out/$w.log; exit 1; }
  grep '^{' $out/$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w', d['n_gpus'], d.get('folded_ranks'), round(d['ms_per_step'],4), d['value'], 'cpu' in str(d.get('cpu_baseline')))"
done
