#!/bin/bash
# Per-shard kernel time (scripts/shard_probe.py) at N = 1 and 8 for work-claim floors (RTAMD_BATCH_FLOOR).
# usage: FLOORS="0 16 64" scripts/floor_probe.sh [shard_probe args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
probe() { timeout -k 10 300 python scripts/shard_probe.py --shards 1 8 --reps 2 "$@" 2>/dev/null | grep "N=" | sed 's/per-shard //; s/, ideal [0-9.]* ms//' | tr '\n' ' '; echo; }
for i in 1 2; do
  for f in ${FLOORS:-0 4 16 64}; do echo "floor $f: $(RTAMD_BATCH_FLOOR=$f probe "$@")"; done
done
