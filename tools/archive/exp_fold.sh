#!/bin/bash
# Fold kernels on the GPU box: parity tests, a batch / width sweep of
# tools/fold_bench (built in-tree beforehand), the r02 kernel beside it, and
# PMC passes.  Output under gpurun_out/fold/.
set -o pipefail
out=gpurun_out/fold; mkdir -p $out; rm -f $out/sweep.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fold.py tests/test_gpu_pir.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for b in 1 4 8 16 17 32 64 128 256; do
  timeout -k 10 120 tools/fold_bench $b 32 24 >> $out/sweep.jsonl || exit 1
done
timeout -k 10 120 tools/bin/fold_bench_r02 64 32 24 >> $out/sweep.jsonl || exit 1
timeout -k 10 120 tools/bin/fold_bench_r02 256 32 24 >> $out/sweep.jsonl || exit 1
for r in 64 128 256; do
  timeout -k 10 120 tools/fold_bench 64 $r 22 >> $out/sweep.jsonl || exit 1
  timeout -k 10 120 tools/fold_bench 16 $r 22 >> $out/sweep.jsonl || exit 1
done
timeout -k 10 120 tools/fold_bench 64 96 22 >> $out/sweep.jsonl || exit 1
cat $out/sweep.jsonl
[ -n "$PROF" ] && bash tools/prof_fold.sh $out/pmc new64=tools/fold_bench:"64 32 24" r02=tools/bin/fold_bench_r02:"64 32 24" new16=tools/fold_bench:"16 32 24" new256=tools/fold_bench:"256 32 24"
exit 0
