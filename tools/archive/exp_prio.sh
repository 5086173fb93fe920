#!/bin/bash
# Wave-priority schemes (DPF_PRIO_STEPS 0-3, dpf_kernels.hip prio_step):
# per-wave finish spread (tools/wave_times.hip) and bench A/B
# on configs[1] and configs[4], all on one box.
set -o pipefail
mkdir -p gpurun_out/prio_wt
for s in 1 3; do
  for shape in "4096 20" "64 24"; do
    # shellcheck disable=SC2086
    WAVE_TIMES_CSV=gpurun_out/prio_wt/s${s}_${shape// /_}.csv timeout -k 10 120 tools/bin/wave_times_s$s $shape | sed "s/^{/{\"scheme\": $s, /" || exit 1
  done
done
timeout -k 10 120 tools/bin/wave_times 4096 20 | sed 's/^{/{"scheme": 0, /' || exit 1
timeout -k 10 400 bash tools/exp_wl.sh prio_s evalfull base prio0 || exit 1
timeout -k 10 400 bash tools/exp_wl.sh prio_s_pir pir base prio0 || exit 1
