#!/bin/bash
# r05: fold parity tests, then the LDS-only barrier vs __syncthreads() on the
# fold microbenchmark (B = 64 / 256, 2^24 and 2^21 records) and on the PIR
# step (variant syncbar), plus the fold ablations.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_fbar2}"; mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fold.py \
   tests/test_gpu_per_rank.py tests/test_gpu_pir.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
bash tools/archive/r05_fbar.sh "$(basename $OUT)"
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
for r in 1 2 3; do
  for w in 1 8; do
    for L in dpf-go_amd/lib/libdpf_hip.so dpf-go_amd/lib/variants/libdpf_hip_syncbar.so; do
      DPF_LIB="$REPO/$L" timeout -k 10 120 python3 bench.py $C --workload pir --emulate-world $w > "$OUT/pir.log" 2>&1 || { echo "FAIL pir"; tail -3 "$OUT/pir.log"; exit 1; }
      grep '^{' "$OUT/pir.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$r W=$w $(basename $L .so)', round(d['ms_per_step'],4), 'fold', k['fold']['kernel_ms'])" | tee -a "$OUT/pir.txt"
    done
  done
done
