#!/bin/bash
# configs[1] strong-scaling per-rank shapes (4096/N keys on one GPU) at forced
# subtree depths D (DPF_SUBTREE_DEPTH) against the depth model's choice.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04strong}"
mkdir -p "$OUT"
for nk in 512 1024 2048; do
  for d in auto 7 6 5 4 3; do
    if [ "$d" = auto ]; then unset DPF_SUBTREE_DEPTH; else export DPF_SUBTREE_DEPTH=$d; fi
    timeout -k 10 120 python bench.py --nkeys $nk --steps 100 --warmup 10 --no-workloads --no-variants --no-api \
        --no-cpu-baseline > "$OUT/nk${nk}_d$d.log" 2>&1
    rc=$?; [ $rc -le 1 ] || { echo "nk $nk d $d rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/nk${nk}_d$d.log') if l.startswith('{')][-1]); r=d['roofline']; print('$nk', '$d', round(d['ms_per_step'],4), r['kernel_ms'], round(d['value']/1e12,3), r['frac'])"
  done
done
unset DPF_SUBTREE_DEPTH
echo done
