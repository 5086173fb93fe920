#!/bin/bash
# Host Gen A/B on the GPU box's CPU: tools/bin/gen_bench (current host_gen)
# vs tools/bin/gen_bench_old (previous build), alternating, logN 20 and 24.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-gen}"
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in gen_bench_old gen_bench; do
    for n in 20 24; do
      timeout -k 5 60 ./tools/bin/$v $n 16 300000 > "$OUT/${v}_${n}_$r.json" || exit 1
      echo "$v r$r $(cat "$OUT/${v}_${n}_$r.json")"
    done
  done
done
