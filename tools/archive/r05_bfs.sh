#!/bin/bash
# r05: breadth-first finish of the shared walk (DPF_COOP_BFS, product) vs one
# walk per thread (variant nobfs) at the small per-rank shapes: parity tests,
# then interleaved bench lines.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_bfs}"; mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_per_rank.py \
   tests/test_gpu_parity.py tests/test_gpu_api.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
declare -A SH
SH[pir8]="--workload pir --emulate-world 8"
SH[pir4]="--workload pir --emulate-world 4"
SH[pir1]="--workload pir"
SH[split8]="--workload split --emulate-world 8"
SH[strong8]="--strong --nkeys 4096 --emulate-world 8"
SH[cfg1]=""
for r in 1 2 3; do
  for s in pir8 pir4 pir1 split8 strong8 cfg1; do
    for L in dpf-go_amd/lib/libdpf_hip.so dpf-go_amd/lib/variants/libdpf_hip_${VAR:-nobfs}.so; do
      tag=$(basename $L .so)
      DPF_LIB="$REPO/$L" timeout -k 10 120 python3 bench.py $C ${SH[$s]} > "$OUT/${s}_${tag}_$r.log" 2>&1 || { echo "FAIL $s $L"; tail -3 "$OUT/${s}_${tag}_$r.log"; exit 1; }
      grep '^{' "$OUT/${s}_${tag}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$r $s $tag', round(d['ms_per_step'],4), 'ms kernel', d['roofline'].get('kernel_ms'))"
    done
  done
done
