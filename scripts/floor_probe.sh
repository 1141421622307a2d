#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
probe() { timeout -k 10 100 python scripts/shard_probe.py --shards 1 8 --reps 2 2>/dev/null | grep "N=" | sed 's/per-shard //; s/, ideal [0-9.]* ms//' | tr '\n' ' '; echo; }
for i in 1 2; do
  for f in ${FLOORS:-0 4 16 64}; do echo "floor $f: $(RTAMD_BATCH_FLOOR=$f probe)"; done
done
