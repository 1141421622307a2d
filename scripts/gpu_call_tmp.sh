# round 6: a second postponed leaf per lane (RT_LEAF_Q=1, _var_lq) against the tree: image hashes, then C2 and C5 timing
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for d in . _var_lq _var_lq2; do
  (cd $d && timeout -k 10 120 python -u scripts/img_hash.py --config c2 --spp 16 && timeout -k 10 120 python -u scripts/img_hash.py --config c5 --spp 2 && timeout -k 10 120 python -u scripts/img_hash.py --config c4 --spp 4) >> gpurun_out/r6_lq_hash.log 2>&1
  rc=$?; echo "hash $d rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u scripts/ab.py time --reps 3 . _var_lq _var_lq2 > gpurun_out/r6_ab_c2_lq.log 2>&1
rc=$?; echo "ab2 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 500 python -u scripts/ab.py time --bench="--config c5 --spp 64" --reps 2 . _var_lq _var_lq2 > gpurun_out/r6_ab_c5_lq.log 2>&1
echo "ab5 rc=$?"
