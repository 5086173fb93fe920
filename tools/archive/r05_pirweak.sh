#!/bin/bash
# PIR per-rank shapes in the weak form: B queries per GPU (total batch B x N),
# rank 0's share (prefix log2(N) bits of every key, DB slice 1/N) timed on 1 GPU.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-pirweak}"; mkdir -p "$OUT"
for spec in "1 64" "2 128" "4 256" "8 512" "8 64" "4 64"; do
  set -- $spec
  timeout -k 10 180 python3 bench.py --workload pir --emulate-world $1 --batch $2 --steps 50 --warmup 10 \
      --no-cpu-baseline --no-sweep --no-api > "$OUT/w$1_b$2.log" 2>&1 || { echo "w$1 b$2 failed"; exit 1; }
  python3 - "$OUT/w$1_b$2.log" <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(ln)
k = d["kernels"]
print(sys.argv[1].split("/")[-1], "ms", round(d["ms_per_step"], 4), "q/s", round(d["value"]), "tree", k["tree"]["kernel_ms"], "fold", k["fold"]["kernel_ms"])
PY
done
