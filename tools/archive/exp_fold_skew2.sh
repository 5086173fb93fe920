#!/bin/bash
# DPF_FOLD_SKEW 50 vs 62 on the other two-workgroups-per-CU fold shapes
# (64- and 128-byte records, 17 and 64 keys), 2 interleaved rounds.
set -o pipefail
out=gpurun_out/fold_skew2; mkdir -p $out; rm -f $out/sweep.jsonl
for r in 1 2; do
  for shape in "64 64 22" "64 128 22" "17 32 24" "48 64 22"; do
    for k in 50 62; do
      # shellcheck disable=SC2086
      DPF_FOLD_SKEW=$k timeout -k 10 120 tools/fold_bench $shape | sed "s/^{/{\"skew\": $k, \"round\": $r, /" >> $out/sweep.jsonl || exit 1
    done
  done
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
