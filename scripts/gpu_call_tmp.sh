# round 6: the step-profile test, C4 scheduling knobs re-swept on the final build
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scenes.py -m gpu -v --timeout 120 --timeout-method thread -rA -s -k step_profile > gpurun_out/r6_gpu_stepprof.log 2>&1
rc=$?; echo "test rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python -u scripts/ab.py time --bench="--config c4 --spp 100" --reps 2 . .:RTAMD_BOX_FIRST=2 .:RTAMD_BOX_FIRST=8 .:RTAMD_TRAV_STOP=4 .:RTAMD_TRAV_STOP=12 > gpurun_out/r6_ab_c4_knobs.log 2>&1
echo "ab rc=$?"
