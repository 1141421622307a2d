mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_bands.py -m gpu -v --timeout 300 --timeout-method thread -rA -s -k "nan_rays or closest_hits or walks_output or bands or grazing or scene_library or cornell" > gpurun_out/r6_gpu6.log 2>&1
rc=$?; echo "tests rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/ab.py time --bench="--config c4 --spp 100" --reps 2 --work . _var_nopre _var_nofilt > gpurun_out/r6_ab_c4_pre.log 2>&1
rc=$?; echo "ab4 rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab.py time --bench="--config c3 --spp 300" --reps 2 . _var_nopre > gpurun_out/r6_ab_c3_pre.log 2>&1
echo "ab3 rc=$?"
