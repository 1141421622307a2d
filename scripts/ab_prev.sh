#!/bin/bash
# Same-box A/B: _ab_prev/ (scripts/ab_prev_build.sh) vs the working tree, C2 kernel time at N = 1
# and per shard at N = 8 (scripts/shard_probe.py), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
probe() { timeout -k 10 100 python scripts/shard_probe.py --shards 1 8 --reps 2 "$@" 2>/dev/null | grep "N=" | sed 's/per-shard //; s/, ideal [0-9.]* ms//' | tr '\n' ' '; echo; }
for i in 1 2; do
  echo "prev: $(cd _ab_prev && probe "$@")"
  echo "new:  $(probe "$@")"
done
