#!/bin/bash
# Compile ONE render-kernel instantiation for register / scratch experiments (seconds instead of the
# whole library) and print its resource usage; --isa FILE also writes its gfx950 assembly.
# usage: scripts/kdev.sh '<explicit instantiation>' [--isa FILE] [extra hipcc flags...]
#   e.g. scripts/kdev.sh 'render_philox2<559u, 3>(RenderArgs, int)' --isa /tmp/c4.s
set -eo pipefail
root=${KDEV_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}  # (KDEV_ROOT: another source tree, e.g. /tmp/ab_src_NAME)
inst=$1; shift
isa=""
if [ "${1:-}" = "--isa" ]; then isa=$2; shift 2; fi
tmp=$(mktemp -d)
printf '#include "rt_kernels.h"\nnamespace {\ntemplate __global__ void %s;\n}\n' "$inst" > "$tmp/k.hip"
flags=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I"$root/include"
       -I"$root/ray-tracing_amd/csrc" -Wno-unused-function "$@")
/opt/rocm/bin/hipcc "${flags[@]}" --cuda-device-only -c -o "$tmp/k.o" "$tmp/k.hip" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill" | sed "s/.*remark: *//; s/ \[-Rpass.*//" | tail -6 | tr "\n" " "; echo
[ -n "$isa" ] && /opt/rocm/bin/hipcc "${flags[@]}" --cuda-device-only -S -o "$isa" "$tmp/k.hip"
rm -rf "$tmp"
