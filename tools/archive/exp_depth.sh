set -uo pipefail
mkdir -p gpurun_out/exp1
for d in 7 6 5; do
  DPF_SUBTREE_DEPTH=$d timeout -k 10 200 python bench.py --workload pir --steps 20 --warmup 5 > gpurun_out/exp1/pir_d$d.log 2>&1 || exit 1
  DPF_SUBTREE_DEPTH=$d timeout -k 10 200 python bench.py --workload split --emulate-world 8 --steps 20 --warmup 5 > gpurun_out/exp1/split8_d$d.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --workload pir --steps 20 --warmup 5 --check > gpurun_out/exp1/pir_auto.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload split --steps 20 --warmup 5 --check > gpurun_out/exp1/split1_auto.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload split --emulate-world 8 --steps 20 --warmup 5 > gpurun_out/exp1/split8_auto.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_pir.py -q -x > gpurun_out/exp1/pir_tests.log 2>&1; tail -2 gpurun_out/exp1/pir_tests.log
for f in gpurun_out/exp1/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"kernel_ms": [0-9.]*' $f)"; done
