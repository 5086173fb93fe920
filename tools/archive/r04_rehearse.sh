#!/bin/bash
# r04 GPU pass: the GPU suite (no -x: every new per-rank test reports), the
# default bench line (driver command, now with the configs[2..4] sub-lines),
# folded --gpus 4 / 8 rehearsals of all four workloads with --check (8 ranks
# on one GPU over gloo: the N=8 code path, not an 8-GPU rate), and the
# configs[1] strong-scaling per-rank shapes (--strong --emulate-world N).
# A crash / timeout (rc >= 124 or a signal) ends the call; test failures do not.
set -uo pipefail
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$REPO"
OUT="gpurun_out/${1:-r04a}"
mkdir -p "$OUT"
step() {   # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep '^{' "$OUT/$name.log" | tail -1 | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a "$name" = tests ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step tests 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
tail -3 "$OUT/tests.log"
step bench_default 400 python bench.py --steps 20 --warmup 5
for n in 4 8; do
  step g${n}_evalfull 500 python bench.py --gpus $n --steps 20 --warmup 5 --check --cpu-seconds 4
  for w in split pir eval; do
    step g${n}_$w 500 python bench.py --gpus $n --workload $w --steps 20 --warmup 5 --check --no-sweep --cpu-seconds 4
  done
done
for w in 2 4 8; do
  step strong_e$w 200 python bench.py --strong --nkeys 4096 --emulate-world $w --steps 50 --warmup 10 \
      --no-variants --no-api --no-cpu-baseline
done
export TMPDIR=/tmp
for w in 1 8; do
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$REPO/$OUT/kt_strong$w" -o kt --output-format csv -- \
      python3 "$REPO/bench.py" --strong --nkeys 4096 --emulate-world $w --steps 50 --warmup 10 --no-variants --no-api \
      --no-cpu-baseline > "$REPO/$OUT/kt_strong$w.log" 2>&1 ) ; echo "kt_strong$w rc=$?"
done
echo done
