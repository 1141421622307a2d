mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/step_profile.py --config c5 --spp 16 > gpurun_out/r6_step_profile_c5.txt 2>&1
rc=$?; echo "sp5 rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/step_profile.py --config c4 --spp 32 > gpurun_out/r6_step_profile_c4.txt 2>&1
rc=$?; echo "sp4 rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/step_profile.py --config c2 --spp 50 > gpurun_out/r6_step_profile_c2.txt 2>&1
rc=$?; echo "sp2 rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/ab.py time --bench="--config c5 --spp 64" --reps 2 . .:RTAMD_LEAF_STOP=8 .:RTAMD_LEAF_STOP=24 .:RTAMD_LEAF_STOP=32 .:RTAMD_TRAV_STOP=8 .:RTAMD_TRAV_STOP=24 > gpurun_out/r6_ab_c5_stops.log 2>&1
rc=$?; echo "ab5 rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab.py time --bench="--config c2" --reps 2 . .:RTAMD_WAVES=3 > gpurun_out/r6_ab_c2_waves.log 2>&1
echo "ab2 rc=$?"
