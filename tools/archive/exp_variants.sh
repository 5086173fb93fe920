#!/bin/bash
# A/B of tree-kernel build variants (tools/build_variant.sh) on the default
# workload, interleaved over 2 rounds, plus one WRITE_SIZE pass per variant.
#   tools/exp_variants.sh <out_tag> <variant>...   ("base" = product build)
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/$1"; shift
mkdir -p "$OUT"
B=(--steps 50 --warmup 10 --spinup 0.5 --no-cpu-baseline --no-variants --no-api --aes ttable)
lib() { if [ "$1" = base ]; then echo "$REPO/dpf-go_amd/lib/libdpf_hip.so"; elif [ -f "$REPO/tools/bin/libdpf_hip_$1.so" ]; then echo "$REPO/tools/bin/libdpf_hip_$1.so"; else echo "$REPO/dpf-go_amd/lib/variants/libdpf_hip_$1.so"; fi; }
for r in 1 2; do
  for v in "$@"; do
    DPF_LIB=$(lib $v) timeout -k 10 200 python bench.py "${B[@]}" --check > "$OUT/${v}_$r.log" 2>&1 || { echo "FAIL $v"; tail -5 "$OUT/${v}_$r.log"; exit 1; }
    grep '^{' "$OUT/${v}_$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v r$r', round(d['ms_per_step'],4), 'kernel_ms', r['kernel_ms'], 'G_aes', round(r['aes_blocks_per_s']/1e9,2))"
  done
done
export TMPDIR=/tmp
for v in "$@"; do
  ( cd /tmp && DPF_LIB=$(lib $v) timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$REPO/$OUT/w_$v" -o w --output-format csv -- \
      python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-variants --no-api --aes ttable > "$REPO/$OUT/w_$v.log" 2>&1 ) || { echo "pmc FAIL $v"; exit 1; }
  python3 - "$REPO/$OUT/w_$v" "$v" <<'EOF'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
acc = collections.defaultdict(list)
for r in rows:
    if "k_evalfull<7" in r.get("Kernel_Name", ""):
        acc[r["Kernel_Name"][:40]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(sys.argv[2], k, "WRITE_SIZE per launch (KB)", round(sum(v) / len(v) * 1.0, 1), "ratio", round(sum(v) / len(v) * 1024 / 536870912, 3))
EOF
done
