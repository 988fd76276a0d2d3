#!/bin/bash
# Host-only AddressSanitizer + UndefinedBehaviorSanitizer build of the kernels' launch planners
# (no device code is compiled; nothing touches a GPU), then run the checks.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
CSRC="$ROOT/realtime_semantic_segmentation_pytorch_amd/csrc"
OUT="${1:-/tmp/rtseg_sanitize}"
mkdir -p "$OUT"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="-O1 -g -std=c++20 --offload-arch=gfx950 --cuda-host-only -fgpu-rdc -I $CSRC/include"
objs=()
for k in conv_igemm conv_halo bn_act dwconv gate act augment detail_loss kd_metrics; do
  /opt/rocm/bin/hipcc -c $FLAGS $SAN "$CSRC/kernels/$k.hip" -o "$OUT/$k.o" &
  objs+=("$OUT/$k.o")
done
wait
/opt/rocm/bin/hipcc -c -x hip $FLAGS $SAN "$ROOT/tools/sanitize/host_plan_check.cpp" -o "$OUT/check.o"
/opt/rocm/bin/hipcc $SAN --offload-arch=gfx950 -fgpu-rdc "$OUT/check.o" "${objs[@]}" -o "$OUT/host_plan_check"
ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_plan_check"
