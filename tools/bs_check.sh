#!/bin/bash
# GPU check of the byte-sliced back end: its parity tests, then the
# configs[1] bench (both back ends) and configs[4] PIR with each, and the
# raw AES-MMO rates.  Usage: tools/bs_check.sh [tag]
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bs1}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bitsliced.py tests/test_gpu_pir.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "bs tests rc=$rc"; tail -4 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['aes_variants'])); print(d['value'])"
[ $rc -eq 0 ] || exit $rc
for impl in ttable bitsliced; do
  timeout -k 10 300 python bench.py --workload pir --aes $impl --steps 20 --warmup 5 > $OUT/pir_$impl.log 2>&1
  rc=$?; echo "pir $impl rc=$rc"; grep '^{' $OUT/pir_$impl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python tools/aes_rates.py > $OUT/aes_rates.json 2>$OUT/aes_rates.err; echo "aes rc=$?"; cat $OUT/aes_rates.json
