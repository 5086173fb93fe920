#!/bin/bash
# Small-batch EvalFull time per forced subtree depth, then the automatic choice.
set -uo pipefail
mkdir -p gpurun_out/lat
for d in 0 1 2 3 4 5 6 7 auto; do
  if [ $d = auto ]; then unset DPF_SUBTREE_DEPTH; else export DPF_SUBTREE_DEPTH=$d; fi
  timeout -k 10 120 python tools/latency.py > gpurun_out/lat/d$d.json 2>/dev/null || exit 1
  cat gpurun_out/lat/d$d.json
done
