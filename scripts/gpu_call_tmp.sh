# round 6: the C4 tail length at 8 shards again, three repetitions
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 800 python -u scripts/ab.py time --bench="--config c4" --shards 1 8 --reps 3 . .:RTAMD_TAIL=1536 .:RTAMD_TAIL=1024 > gpurun_out/r6_ab_c4_tail2.log 2>&1
echo "ab rc=$?"
