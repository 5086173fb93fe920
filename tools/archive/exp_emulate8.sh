#!/bin/bash
# N=8 per-rank shapes on one GPU: kernel breakdown (rocprofv3) and the
# subtree depth (DPF_SUBTREE_DEPTH) for split and PIR.
set -o pipefail
out=gpurun_out/emulate8; mkdir -p $out
B="--emulate-world 8 --steps 30 --warmup 5 --no-cpu-baseline --no-variants --no-api --no-sweep"
for w in split pir; do
  for d in auto 3 4 5 6; do
    if [ $d = auto ]; then unset DPF_SUBTREE_DEPTH; else export DPF_SUBTREE_DEPTH=$d; fi
    timeout -k 10 120 python bench.py --workload $w $B > $out/${w}_d$d.log 2>&1 || { tail -5 $out/${w}_d$d.log; exit 1; }
    grep '^{' $out/${w}_d$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w D=$d', round(d['ms_per_step'],4), 'kernels', d['roofline']['kernel_ms'])"
  done
  unset DPF_SUBTREE_DEPTH
done
export TMPDIR=/tmp
for w in split pir; do
  ( cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/kt_$w" -o kt --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w $B > "$GRAFT_REPO_ROOT/$out/kt_$w.log" 2>&1 ) || { echo "kt $w failed"; exit 1; }
  python3 - "$out/kt_$w" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
