#!/bin/bash
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/bs1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bitsliced.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "bs tests rc=$rc"; tail -12 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['aes_variants'], indent=1)); print(d['value'])"
timeout -k 10 120 python tools/aes_rates.py > $OUT/aes_rates.json 2>$OUT/aes_rates.err; echo "aes rc=$?"; cat $OUT/aes_rates.json
