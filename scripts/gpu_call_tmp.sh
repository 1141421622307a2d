# round 6: rare-fallback branches marked unlikely (RT_COLD_BRANCHES=1, _var_cold) against the tree: hashes, C4, C5, C2
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for d in . _var_cold; do
  (cd $d && timeout -k 10 120 python -u scripts/img_hash.py --config c4 --spp 4 && timeout -k 10 120 python -u scripts/img_hash.py --config c2 --spp 8) >> gpurun_out/r6_cold_hash.log 2>&1
  rc=$?; echo "hash $d rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u scripts/ab.py time --bench="--config c4 --spp 100" --reps 3 . _var_cold > gpurun_out/r6_ab_cold.log 2>&1
rc=$?; echo "ab4 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u scripts/ab.py time --bench="--config c5 --spp 64" --reps 2 . _var_cold >> gpurun_out/r6_ab_cold.log 2>&1
rc=$?; echo "ab5 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u scripts/ab.py time --reps 2 . _var_cold >> gpurun_out/r6_ab_cold.log 2>&1
echo "ab2 rc=$?"
