#!/bin/bash
# r05: the PIR step eager vs captured in a HIP graph (tools/pir_graph.py) at
# the N = 8 / 4 rank shapes and on one GPU.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_graph}"; mkdir -p "$OUT"
for pb in 3 2 0; do
  PB=$pb timeout -k 10 120 python3 tools/pir_graph.py 400 > "$OUT/graph_pb$pb.log" 2>&1 || { echo "graph pb=$pb failed"; tail -8 "$OUT/graph_pb$pb.log"; exit 1; }
  echo "pb=$pb $(tail -1 "$OUT/graph_pb$pb.log")" | tee -a "$OUT/graph.txt"
done
