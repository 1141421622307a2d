cd $GRAFT_REPO_ROOT
probe() { timeout -k 10 100 python scripts/shard_probe.py --shards 1 2 4 8 --reps 2 2>/dev/null | grep "N=" | sed 's/per-shard //; s/, ideal [0-9.]* ms//' | tr '\n' ' '; echo; }
echo "prev: $(cd _ab_prev && probe)"
for b in 128 256 64; do echo "batch $b: $(RTAMD_BATCH=$b probe)"; done
