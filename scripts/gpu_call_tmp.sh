# round 6: C2's tile order reversed (RTAMD_TILE_REV=1: the slab's tiles last to first, the sky rows last) at 1 and 8 shards
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab.py time --bench="--config c2" --shards 1 8 --reps 3 . .:RTAMD_TILE_REV=1 > gpurun_out/r6_ab_c2_rev.log 2>&1
echo "ab rc=$?"
