#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the XOR fold for wide records (tools/fold_bench
# <nkeys> <rec_bytes> <log2 nrec>), one PMC pass per counter.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/${1:-gpurun_out/foldwide}"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
for cfg in "64 32 24" "64 64 22" "64 128 22" "64 256 22" "16 128 22" "64 96 22"; do
  tag=$(echo $cfg | tr ' ' _); mkdir -p "$OUT/$tag"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c -d "$OUT/$tag/$c" -o p --output-format csv -- "$REPO/tools/fold_bench" $cfg \
      > "$OUT/$tag/$c.log" 2>&1 || { echo "fail $tag $c"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = {}
for d in sorted(glob.glob(sys.argv[1] + "/*_*_*")):
    nk, rb, lg = map(int, os.path.basename(d).split("_"))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_fold" in r["Kernel_Name"]:
                acc[r["Kernel_Name"].split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
    nrec = 1 << lg
    alg = nrec * rb + nk * nrec / 8
    for k, v in acc.items():
        f = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"]) * 1024 * 2     # gfx950: FETCH_SIZE reports half of wide streaming reads
        w = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) * 1024
        out[f"{nk}keys_{rb}B"] = {"kernel": k, "fetch_bytes": f, "write_bytes": w, "algorithmic_read_bytes": alg,
                                  "fetch_over_algorithmic": round(f / alg, 4)}
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
