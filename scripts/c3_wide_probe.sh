cd $GRAFT_REPO_ROOT
for e in "" "RTAMD_WIDE=1" "RTAMD_WIDE=1 RTAMD_WAVES=4" "RTAMD_WIDE=1 RTAMD_WAVES=2" "RTAMD_WIDE=1 RTAMD_LEAF_LDS=0"; do
  echo "== $e"
  env $e timeout -k 10 120 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-work 2>&1 | grep -o '"value": [0-9.]*, "unit"\|kernel [0-9.]* ms' | tr '\n' ' '; echo
done
