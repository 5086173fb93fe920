#!/bin/bash
# Batched Eval variants at configs[2] (HBM frontier default, LDS frontier, plain root walks).
set -uo pipefail
mkdir -p gpurun_out/exp2
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/exp2/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/exp2/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for m in hbm lds plain; do
  DPF_EVAL_MODE=$m timeout -k 10 300 python bench.py --workload eval --steps 20 --warmup 5 --check \
      > gpurun_out/exp2/eval_$m.log 2>&1 || exit 1
  echo "$m $(grep -o '"value": [0-9.e+]*' gpurun_out/exp2/eval_$m.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp2/eval_$m.log)"
done
