cd $GRAFT_REPO_ROOT
for i in 1 2; do
for lib in dpf-go_amd/lib/libdpf_hip.so dpf-go_amd/lib/variants/libdpf_hip_fold_r01.so; do
  DPF_LIB=$lib timeout -k 10 200 python bench.py --workload pir --steps 30 --warmup 5 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1
done; done
