#!/bin/bash
# Per-wave start/end of the tree kernel (tools/wave_times.hip, built in-tree
# into tools/bin/wave_times) at the configs[1] shape and the PIR tree's shape
# (64 keys at logN 24), three launches each.  gpurun_out/wt/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/wt
mkdir -p $O
for r in 1 2 3; do
  WAVE_TIMES_CSV=$O/c1_$r.csv timeout -k 10 120 tools/bin/wave_times 4096 20 | sed 's/^{/{"shape": "configs[1]", /' >> $O/summary.jsonl || exit $?
  WAVE_TIMES_CSV=$O/pir_$r.csv timeout -k 10 120 tools/bin/wave_times 64 24 | sed 's/^{/{"shape": "pir tree", /' >> $O/summary.jsonl || exit $?
done
