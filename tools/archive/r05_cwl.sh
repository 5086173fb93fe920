#!/bin/bash
# r05: walk correction words staged in LDS (DPF_WALK_CW_LDS=1, product) vs
# scalar loads per level (lib/variants/libdpf_hip_nocwl.so; LIBS picks the
# variants), interleaved,
# at the per-rank shapes where the shared walk is on the critical path and at
# the 1-GPU configs.  Optional: the GPU parity suite first (arg 2 = tests).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_cwl}"; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
# SPECS: "workload:world,..." (default: every per-rank shape and the 1-GPU configs)
IFS=, read -r -a SPEC_LIST <<< "$(echo "${SPECS:-pir:8,pir:4,pir:1,split:8,evalfull-strong:8,evalfull:1}" | tr ':' ' ')"
COMMON="--steps 60 --warmup 10 --no-cpu-baseline --no-sweep --no-api --no-variants --no-workloads"
for r in 1 2; do
  for lib in ${LIBS:-product nocwl}; do
    if [ $lib = product ]; then unset DPF_LIB; else export DPF_LIB=$REPO/dpf-go_amd/lib/variants/libdpf_hip_$lib.so; fi
    for spec in "${SPEC_LIST[@]}"; do
      set -- $spec
      wl=$1; w=$2; extra=""
      if [ $wl = evalfull-strong ]; then wl=evalfull; extra="--strong"; fi
      timeout -k 10 180 python3 bench.py --workload $wl --emulate-world $w $extra $COMMON > "$OUT/run.log" 2>&1 || { echo "$lib $spec failed"; tail -5 "$OUT/run.log"; exit 1; }
      python3 - "$OUT/run.log" "$r $lib $spec" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d.get("kernels", {})
extra = f" tree {k['tree']['kernel_ms']} fold {k['fold']['kernel_ms']}" if "tree" in k else ""
print(sys.argv[2], "ms", round(d["ms_per_step"], 4), extra)
PY
    done
  done
done
