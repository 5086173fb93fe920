#!/bin/bash
# PIR: fold R=8 vs R=16 (interleaved), then per-kernel counters of the default build.
set -uo pipefail
mkdir -p gpurun_out/exp4
for r in 1 2; do
  for v in base fold16; do
    if [ $v = base ]; then unset DPF_LIB; else export DPF_LIB=$PWD/dpf-go_amd/lib/variants/libdpf_hip_$v.so; fi
    timeout -k 10 300 python bench.py --workload pir --steps 30 --warmup 5 --check > gpurun_out/exp4/pir_${v}_$r.log 2>&1 || exit 1
    echo "$v r$r $(grep -o '"value": [0-9.e+]*' gpurun_out/exp4/pir_${v}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp4/pir_${v}_$r.log)"
  done
done
unset DPF_LIB
tools/counters.sh gpurun_out/exp4/cnt pir > /dev/null && python3 -c "
import json; s=json.load(open('gpurun_out/exp4/cnt/summary.json'))
for k,v in s.items():
    if 'avg_ns' in v and v['avg_ns']>10000: print(k, round(v['avg_ns']/1e3,1),'us', 'VALU',v.get('SQ_INSTS_VALU'), 'WAIT_ANY/WAVE', round(v.get('SQ_WAIT_ANY',0)/max(1,v.get('SQ_WAVE_CYCLES',1)),3), 'FETCH', v.get('FETCH_SIZE'), 'WRITE', v.get('WRITE_SIZE'))
"
