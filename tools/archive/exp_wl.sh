#!/bin/bash
# A/B of build variants on one bench workload, 3 interleaved rounds, plus a
# kernel trace per variant.
#   tools/exp_wl.sh <out_tag> <workload> <variant>...   ("base" = product build,
#   others: tools/bin/libdpf_hip_<variant>.so from tools/build_variant.sh)
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/$1"; WL="$2"; shift 2
mkdir -p "$OUT"
B=(--workload "$WL" --steps 30 --warmup 5 --spinup 0.5 --no-cpu-baseline --no-variants --no-api --no-sweep --aes "${AES:-ttable}")
lib() { if [ "$1" = base ]; then echo "$REPO/dpf-go_amd/lib/libdpf_hip.so"; else echo "$REPO/tools/bin/libdpf_hip_$1.so"; fi; }
for r in 1 2 3; do
  for v in "$@"; do
    DPF_LIB=$(lib $v) timeout -k 10 200 python bench.py "${B[@]}" --check > "$OUT/${v}_$r.log" 2>&1 || { echo "FAIL $v"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
    grep '^{' "$OUT/${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v r$r', round(d['ms_per_step'],4), d['value'])"
  done
done
export TMPDIR=/tmp
for v in "$@"; do
  ( cd /tmp && DPF_LIB=$(lib $v) timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/t_$v" -o t --output-format csv -- \
      python3 "$REPO/bench.py" "${B[@]}" --steps 10 --warmup 2 > "$REPO/$OUT/t_$v.log" 2>&1 ) || { echo "trace FAIL $v"; exit 1; }
  python3 - "$REPO/$OUT/t_$v" "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(sys.argv[2], r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
