# round 6: the global spheres kernel from its own unit (cold-branch hints) against the spheres unit's (RTAMD_NO_COLD=1)
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
( timeout -k 10 120 python -u scripts/img_hash.py --config c5 --spp 2 && RTAMD_NO_COLD=1 timeout -k 10 120 python -u scripts/img_hash.py --config c5 --spp 2 ) > gpurun_out/r6_coldg_hash.log 2>&1
rc=$?; echo "hash rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/ab.py time --bench="--config c5 --spp 64" --reps 3 . .:RTAMD_NO_COLD=1 > gpurun_out/r6_ab_coldg.log 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -ge 124 ] && exit $rc
scripts/gpu_steps.sh gputest_cold 900 "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x"
