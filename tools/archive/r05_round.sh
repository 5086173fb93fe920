#!/bin/bash
# r05 round profile: the GPU parity suite, smoke(), the driver's default bench
# command, a rocprofv3 kernel trace of it, and FETCH_SIZE / WRITE_SIZE passes
# (one counter per run) of every workload for roofline.traffic.
# Usage: tools/archive/r05_round.sh <tag>.  Each GPU step has its own time limit;
# the first failure ends the call.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
TAG="${1:-r05_round}"
OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
t0=$(date +%s)
timeout -k 10 600 python3 bench.py > "$OUT/bench_default.log" 2>&1
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - t0 ))s"; grep '^{' "$OUT/bench_default.log" | tail -1 | cut -c1-400
[ $rc -eq 0 ] || exit $rc
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --steps 40 --warmup 5 --no-cpu-baseline > "$REPO/$OUT/kt.log" 2>&1 )
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f "$OUT"/kt/*kernel_trace.csv
for wl in evalfull eval split pir; do
  for c in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $c -d "$REPO/$OUT/pmc_${wl}_$c" -o p --output-format csv -- \
        python3 "$REPO/bench.py" --workload $wl --steps 5 --warmup 2 --spinup 0 --no-cpu-baseline --no-sweep --no-api \
        --no-variants --no-workloads > "$REPO/$OUT/pmc_${wl}_$c.log" 2>&1 ) || { echo "pmc $wl $c failed"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
for wl in ("evalfull", "eval", "split", "pir"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"{out}/pmc_{wl}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                if k.startswith("dpfk::"):
                    k = k[6:]
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, v in acc.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            fb = sorted(v["FETCH_SIZE"])[len(v["FETCH_SIZE"]) // 2] * 1024 * 2   # gfx950: reads count half
            wb = sorted(v["WRITE_SIZE"])[len(v["WRITE_SIZE"]) // 2] * 1024
            res[k] = {"fetch_bytes": fb, "write_bytes": wb, "traffic_bytes": fb + wb}
    name = "traffic.json" if wl == "evalfull" else f"traffic_{wl}.json"
    json.dump(res, open(os.path.join(out, name), "w"), indent=1, sort_keys=True)
    print(wl, {k: round(x["traffic_bytes"] / 1e6, 2) for k, x in res.items()})
PY
