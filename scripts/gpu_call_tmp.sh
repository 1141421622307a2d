# round 6: the 8-wide tree as record pairs (RTAMD_W8=1, A/B): image hashes against the default, then C5 timing
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
mkdir -p gpurun_out
( timeout -k 10 120 python -u scripts/img_hash.py --config c5 --spp 2 && RTAMD_W8=1 timeout -k 10 120 python -u scripts/img_hash.py --config c5 --spp 2 && \
  timeout -k 10 120 python -u scripts/img_hash.py --config c2 --spp 8 && RTAMD_W8=1 timeout -k 10 120 python -u scripts/img_hash.py --config c2 --spp 8 ) > gpurun_out/r6_w8_hash.log 2>&1
rc=$?; echo "hash rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u scripts/ab.py time --bench="--config c5 --spp 64" --reps 2 . .:RTAMD_W8=1 > gpurun_out/r6_ab_c5_w8.log 2>&1
echo "ab5 rc=$?"
