# round 6: the W8 render test
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scenes.py -m gpu -v --timeout 200 --timeout-method thread -rA -s -k "w8" > gpurun_out/r6_gpu_w8b.log 2>&1
echo "tests rc=$?"
