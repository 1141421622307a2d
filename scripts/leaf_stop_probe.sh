#!/bin/bash
# Kernel time of one config under several RTAMD_LEAF_STOP values (binary/4-wide postponed leaves).
# usage: scripts/leaf_stop_probe.sh "<bench args>" v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
args=$1; shift
for v in "$@"; do
  echo "leaf_stop=$v: $(RTAMD_LEAF_STOP=$v timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work $args 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' ')"
done
