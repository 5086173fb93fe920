#!/bin/bash
# r05 end of round: kernel traces of the emulated per-rank steps (PIR at
# N = 8 and 4, configs[3] split at N = 8) on the final code.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_kt_ranks}"; mkdir -p "$OUT"
export TMPDIR=/tmp
C="--steps 100 --warmup 10 --no-cpu-baseline --no-api --no-variants --no-sweep --no-workloads"
for spec in "pir 8" "pir 4" "split 8"; do
  set -- $spec
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_$1_$2" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" --workload $1 --emulate-world $2 $C > "$REPO/$OUT/kt_$1_$2.log" 2>&1 ) || { echo "kt $spec failed"; exit 1; }
  rm -f "$OUT"/kt_$1_$2/*kernel_trace.csv
  echo "== $spec"; grep '^{' "$OUT/kt_$1_$2.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step ms', round(d['ms_per_step'],4))"
  python3 - "$OUT/kt_$1_$2/kt_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(" ", r["Name"].split("(")[0][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
