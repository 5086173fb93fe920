#!/bin/bash
# configs[4] PIR line: matrix-core fold over the sliced DB vs the LDS fold, interleaved, with the batch sweep.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04pir}"
mkdir -p "$OUT"
for r in 1 2; do
  for f in mfma lds; do
    timeout -k 10 300 python bench.py --workload pir --pir-fold $f --steps 30 --warmup 5 --check --no-cpu-baseline \
        > "$OUT/pir_${f}_$r.log" 2>&1
    rc=$?; [ $rc -le 1 ] || { echo "pir $f rc=$rc"; exit $rc; }
    python3 -c "
import json; d=json.loads([l for l in open('$OUT/pir_${f}_$r.log') if l.startswith('{')][-1])
k=d['kernels']; print('$f r$r', round(d['ms_per_step'],4), 'tree', k['tree']['kernel_ms'], 'fold', k['fold']['kernel_ms'],
      {b: v['ms_per_step'] for b, v in d.get('batch_sweep', {}).items()})"
  done
done
