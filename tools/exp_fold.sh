#!/bin/bash
# Builds (here) / runs (GPU box) the fold microbenchmark variants.
#   tools/exp_fold.sh build   -> tools/fold_bench_e{0,1,2,3}
#   tools/exp_fold.sh run     -> one JSON line per variant
set -euo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
if [ "${1:-run}" = build ]; then
  for e in 0 1 2 3; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDPF_FOLD_EXP=$e "$REPO/tools/fold_bench.hip" -o "$REPO/tools/fold_bench_e$e" &
  done
  wait
else
  for e in 0 1 2 3; do timeout -k 10 60 "$REPO/tools/fold_bench_e$e" "${2:-64}"; done
fi
