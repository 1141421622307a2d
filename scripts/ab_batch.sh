cd $GRAFT_REPO_ROOT
probe() { timeout -k 10 100 python scripts/shard_probe.py --shards 1 2 4 8 --reps 2 2>/dev/null | grep "N=" | sed 's/per-shard //; s/, ideal [0-9.]* ms//' | tr '\n' ' '; echo; }
echo "prev: $(cd _ab_prev && probe)"
for cfg in "128 32" "128 16" "128 8" "256 8"; do set -- $cfg
  echo "batch $1 chunk $2: $(RTAMD_BATCH=$1 RTAMD_CHUNK=$2 probe)"
done
