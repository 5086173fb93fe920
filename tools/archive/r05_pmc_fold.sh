#!/bin/bash
# r05: what limits the matrix-core fold k_fold_mfma<2,2,2,1> at configs[4]
# (B = 64, 2^24 x 32 B)?  tools/fold_bench (built in-tree) under one PMC
# group per rocprofv3 run, then a kernel trace.  Counters: VALU work (the FP4
# expansion), MFMA busy, texture addresser / L1 / L2 read requests, and wait
# cycles.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out/${1:-r05_pmc_fold}"; mkdir -p "$OUT"
export TMPDIR=/tmp FOLD_MODE=mfma
cd /tmp
NK=${NK:-64}
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "TA_BUSY_avr TA_TA_BUSY_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_VALU_MFMA_BUSY_CYCLES" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- "$REPO/tools/fold_bench" $NK 32 24 \
      > "$OUT/p$i.log" 2>&1 || echo "pass $i ($grp) failed rc=$?"
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "$REPO/tools/fold_bench" $NK 32 24 \
    > "$OUT/kt.log" 2>&1 || echo "kt failed"
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "k_fold" in k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        out.setdefault("kernel_stats", {})[r["Name"][:60]] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
grep -h '^{' "$OUT"/kt.log | tail -1
