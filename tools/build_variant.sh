#!/bin/bash
# A/B build of libdpf_hip.so with extra preprocessor flags on the tree kernels
# (measurement only; the product build is `make -C dpf-go_amd`).
#   tools/build_variant.sh <name> "-DFOO=1 -DBAR=2" ["flags for dpf_kernels.hip only"]
# -> dpf-go_amd/lib/variants/libdpf_hip_<name>.so  (select with DPF_LIB=...)
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; FLAGS="$2"; KFLAGS="${3:-}"
L="$REPO/dpf-go_amd/lib"
O="$L/variants/$NAME"
mkdir -p "$O"
make -s -C "$REPO/dpf-go_amd" > /dev/null
HIPCC=/opt/rocm/bin/hipcc
CXX=(-O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950)
for f in dpf_kernels bs_kernels pir_kernels dpf_capi; do
  X=""; [ "$f" = dpf_kernels ] && X="$KFLAGS"
  # shellcheck disable=SC2086
  $HIPCC "${CXX[@]}" $FLAGS $X -c "$REPO/dpf-go_amd/csrc/$f.hip" -o "$O/$f.o" &
done
wait
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$L/variants/libdpf_hip_$NAME.so" \
    "$O/dpf_kernels.o" "$O/bs_kernels.o" "$O/pir_kernels.o" "$O/dpf_capi.o" "$L/host_gen.o" "$L/host_eval.o" -lpthread
echo "$L/variants/libdpf_hip_$NAME.so"
