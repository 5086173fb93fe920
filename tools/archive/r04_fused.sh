#!/bin/bash
# Fused PIR kernel (k_pir_fused): parity tests, then the PIR bench line with
# the two-launch kernel and the fused kernel, interleaved.
# Output: gpurun_out/fz/$1/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/fz/${1:-run}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pir_fused.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  DPF_PIR_KERNEL=split timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep --check > $O/pir_split_$i.log 2>&1 || exit $?
  DPF_PIR_KERNEL=fused timeout -k 10 200 python bench.py --workload pir --steps 100 --warmup 10 --no-cpu-baseline --no-sweep --check > $O/pir_fused_$i.log 2>&1 || exit $?
done
