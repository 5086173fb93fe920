#!/bin/bash
# r05: GPU tests of the changed paths, then the configs[4] per-rank profile.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_check}"
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
   tests/test_gpu_fold.py tests/test_gpu_per_rank.py tests/test_gpu_pir_fused.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; grep -E "PASSED|FAILED|SKIPPED" "$OUT/tests.log" | awk '{print $NF}' | sort | uniq -c
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$OUT/tests.log" | head; exit $rc; }
DPF_LIB=dpf-go_amd/lib/variants/libdpf_hip_exp.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
   tests/test_gpu_pir_fused.py > "$OUT/tests_exp.log" 2>&1 || { tail -20 "$OUT/tests_exp.log"; exit 1; }
tail -2 "$OUT/tests_exp.log"
bash tools/archive/r05_pir8.sh r05_pir8
