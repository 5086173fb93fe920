#!/bin/bash
# r05: single-call latency (tools/small_calls.py) with the host's VAES path
# and with AES-NI only (DPF_HOST_ISA=aesni): the measured crossover sets
# the AUTO routing threshold of each host ISA (dpf_capi.hip).
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r05_small}"; mkdir -p "$OUT"
timeout -k 10 300 python3 tools/small_calls.py > "$OUT/small_vaes.json" 2> "$OUT/small_vaes.err" || { tail -5 "$OUT/small_vaes.err"; exit 1; }
DPF_HOST_ISA=aesni timeout -k 10 300 python3 tools/small_calls.py > "$OUT/small_aesni.json" 2> "$OUT/small_aesni.err" || { tail -5 "$OUT/small_aesni.err"; exit 1; }
for f in small_vaes small_aesni; do
  python3 -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', 'isa', d['host_isa'], 'auto', d['auto_max_logN'], 'crossover', d['measured_crossover_logN'], {n: (r['host_ms'], r['gpu_ms']) for n, r in d['evalfull'].items()})"
done
