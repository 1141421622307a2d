#!/bin/bash
# Constant per-launch overhead of the C2 kernel: shard probe at 1, 2 and 8 shards under a few
# settings given as arguments (e.g. RTAMD_BATCH=128; RTAMD_CHUNK changes the summation order:
# timing only). `-` = defaults.
set -e
mkdir -p gpurun_out
out=gpurun_out/tail_probe.txt
: > $out
for cfg in "$@"; do
  [ "$cfg" = "-" ] && cfg=""
  echo "== ${cfg:-default}" >> $out
  env $cfg timeout -k 10 120 python -u scripts/shard_probe.py --shards 1 2 8 --reps 3 >> $out 2>&1
done
grep -v amdgpu.ids $out
