#!/bin/bash
# Deeper shared walk (DPF_COOP_EXTRA = 1, 2 variant libs) vs the product lib,
# interleaved: headline, configs[1] strong per-rank shapes, split and PIR.
# The macro lives in commit 2752386 (dropped after this A/B: neutral);
# build the variants there with tools/build_variant.sh coopN "" -DDPF_COOP_EXTRA=N.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04coopx}"
mkdir -p "$OUT"
V="$REPO/dpf-go_amd/lib/variants"
B=(--steps 50 --warmup 10 --no-cpu-baseline --no-variants --no-api --no-workloads)
run() {   # name lib args...
  local name=$1 lib=$2; shift 2
  DPF_LIB=$lib timeout -k 10 200 python bench.py "${B[@]}" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; [ $rc -le 1 ] || { echo "$name rc=$rc"; exit $rc; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); r=d['roofline']; print('$name', round(d['ms_per_step'],4), r.get('kernel_ms'), round(d['value']/1e12,4))"
}
for r in 1 2; do
  for v in 0 1 2; do
    lib=""; [ $v -gt 0 ] && lib="$V/libdpf_hip_coop$v.so"
    run "full_c${v}_$r" "$lib" --check
    for w in 4 8; do run "strong${w}_c${v}_$r" "$lib" --strong --nkeys 4096 --emulate-world $w; done
    run "split_c${v}_$r" "$lib" --workload split --check
    run "pir_c${v}_$r" "$lib" --workload pir --no-sweep --check
  done
done
