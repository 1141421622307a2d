#!/bin/bash
# Kernel time under RTAMD_TRAV_STOP / RTAMD_LEAF_STOP settings (replacement-loop refill and leaf-step
# thresholds, in 64ths of a wave's live lanes). usage: scripts/stop_sweep.sh "<bench args>" "T:L" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
args=$1; shift
for tl in "$@"; do
  t=${tl%%:*}; l=${tl##*:}
  echo "trav $t leaf $l: $(RTAMD_TRAV_STOP=$t RTAMD_LEAF_STOP=$l timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work $args 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' ')"
done
