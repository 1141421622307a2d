# round 6: opaque Philox key + cold-branch hints (_var_okc) on C4 and C3
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
for d in . _var_okc; do
  (cd $d && timeout -k 10 120 python -u scripts/img_hash.py --config c4 --spp 4 && timeout -k 10 120 python -u scripts/img_hash.py --config c3 --spp 8) >> gpurun_out/r6_okc_hash.log 2>&1
  rc=$?; echo "hash $d rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u scripts/ab.py time --bench="--config c4 --spp 100" --reps 3 . _var_okc > gpurun_out/r6_ab_okc.log 2>&1
rc=$?; echo "ab4 rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u scripts/ab.py time --bench="--config c3 --spp 300" --reps 3 . _var_okc >> gpurun_out/r6_ab_okc.log 2>&1
echo "ab3 rc=$?"
