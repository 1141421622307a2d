# round 6: C2 with cold-branch hints on top of the opaque key (_var_c2cold)
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab.py time --reps 4 . _var_c2cold > gpurun_out/r6_ab_c2cold.log 2>&1
echo "ab rc=$?"
