# round 6: the camera read from the kernarg segment per sample (RT_CAM_KERNARG=1, _var_ck): hashes, C2, C5, C4
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for d in . _var_ck; do
  (cd $d && timeout -k 10 120 python -u scripts/img_hash.py --config c2 --spp 8 && timeout -k 10 120 python -u scripts/img_hash.py --config c4 --spp 4 && timeout -k 10 120 python -u scripts/img_hash.py --config c5 --spp 2) >> gpurun_out/r6_ck_hash.log 2>&1
  rc=$?; echo "hash $d rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u scripts/ab.py time --reps 3 . _var_ck > gpurun_out/r6_ab_ck.log 2>&1
rc=$?; echo "ab2 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u scripts/ab.py time --bench="--config c5 --spp 64" --reps 2 . _var_ck >> gpurun_out/r6_ab_ck.log 2>&1
rc=$?; echo "ab5 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u scripts/ab.py time --bench="--config c4 --spp 100" --reps 3 . _var_ck >> gpurun_out/r6_ab_ck.log 2>&1
echo "ab4 rc=$?"
