# round 6: C3 walks re-measured: binary (default) vs 4-wide (RTAMD_WIDE=1); refill / box-first thresholds
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python -u scripts/ab.py time --bench="--config c3 --spp 300" --reps 2 . .:RTAMD_WIDE=1 .:RTAMD_TRAV_STOP=4 .:RTAMD_TRAV_STOP=16 > gpurun_out/r6_ab_c3_walks.log 2>&1
echo "ab rc=$?"
