B="--workload pir --steps 30 --warmup 5 --no-cpu-baseline --no-variants --no-api --no-sweep"
for d in 4 5 6 7; do
  DPF_SUBTREE_DEPTH=$d timeout -k 10 120 python bench.py $B > gpurun_out/depth_$d.log 2>&1 || exit 1
  grep '^{' gpurun_out/depth_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('D=$d', round(d['ms_per_step'],4), d['roofline']['kernel_ms'])"
done
