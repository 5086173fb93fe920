#!/bin/bash
# Fold kernels with / without issue priority by progress (DPF_FOLD_PRIO),
# 2 interleaved rounds of tools/fold_bench over PIR and payload shapes.
set -o pipefail
out=gpurun_out/fold_prio; mkdir -p $out; rm -f $out/sweep.jsonl
for r in 1 2; do
  for shape in "64 32 24" "4 32 24" "16 128 22" "128 32 24" "256 32 24" "64 128 22"; do
    for b in prio1 prio0; do
      # shellcheck disable=SC2086
      timeout -k 10 120 tools/bin/fold_bench_$b $shape | sed "s/^{/{\"bin\": \"$b\", \"round\": $r, /" >> $out/sweep.jsonl || exit 1
    done
  done
done
python3 - $out/sweep.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line)
    d[(j["nkeys"], j["rec_bytes"], j["bin"])].append((j["fold_us"], j["ok"]))
for k in sorted(d):
    print(*k, d[k])
PY
