#!/bin/bash
# PIR answer pipelined over 2^s subtree slices (tree of slice j+1 beside the
# fold of slice j, two streams): DPF_PIR_SLICES = 0, 1, 2, 3, twice each.
set -uo pipefail
out=gpurun_out/pirslices; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pir.py > $out/tests0.log 2>&1 || { tail -20 $out/tests0.log; exit 1; }
DPF_PIR_SLICES=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pir.py tests/test_gpu_fold.py > $out/tests2.log 2>&1 || { tail -20 $out/tests2.log; exit 1; }
tail -1 $out/tests2.log
for r in 1 2; do for sl in 0 1 2 3; do
  DPF_PIR_SLICES=$sl timeout -k 10 200 python bench.py --workload pir --steps 30 --warmup 5 --no-sweep --check > $out/s${sl}_$r.log 2>&1 || { tail -5 $out/s${sl}_$r.log; exit 1; }
  echo "slices=2^$sl r$r $(grep -o '"ms_per_step": [0-9.]*' $out/s${sl}_$r.log) $(grep -o '"kernel_ms": [0-9.]*' $out/s${sl}_$r.log)"
done; done
