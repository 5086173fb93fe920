#!/bin/bash
# k_fold4r: share of a CU's chunk pair given to its first workgroup
# (DPF_FOLD_SKEW, launch_4r), 2 interleaved rounds of tools/fold_bench, plus
# per-wave times (tools/bin/fold_times) at the chosen shapes.
set -o pipefail
out=gpurun_out/fold_skew; mkdir -p $out; rm -f $out/sweep.jsonl
for r in 1 2; do
  for shape in "64 32 24" "32 32 24" "128 32 24"; do
    for k in 50 55 58 62 66; do
      # shellcheck disable=SC2086
      DPF_FOLD_SKEW=$k timeout -k 10 120 tools/fold_bench $shape | sed "s/^{/{\"skew\": $k, \"round\": $r, /" >> $out/sweep.jsonl || exit 1
    done
  done
done
for k in 50 60; do
  DPF_FOLD_SKEW=$k FOLD_TIMES_CSV=$out/times_$k.csv timeout -k 10 120 tools/bin/fold_times 64 32 24 > /dev/null || exit 1
done
python3 - $out/sweep.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    j = json.loads(line)
    d[(j["nkeys"], j["rec_bytes"], j["skew"])].append((j["fold_us"], j["ok"]))
for k in sorted(d):
    print(*k, d[k])
PY
