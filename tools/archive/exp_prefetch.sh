#!/bin/bash
# A/B of k_fold4r's DB prefetch depth (DPF_FOLD_PREFETCH 1..3) against the
# r03b kernel (tools/ab/pir_kernels_r03b.hip), 2 interleaved rounds of
# tools/fold_bench over PIR and wide-record shapes.
set -o pipefail
out=gpurun_out/prefetch; mkdir -p $out; rm -f $out/sweep.jsonl
for r in 1 2; do
  for shape in "64 32 24" "32 32 24" "128 32 24" "256 32 24" "64 64 22" "64 128 22" "64 256 22"; do
    for b in head p1 p2 p3; do
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
