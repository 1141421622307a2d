# round-6 evidence, part 3: C5 profiles and bench line, the C4 parts probe, shard probes of C2 and C4
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
scripts/gpu_round_profiles.sh r6 c5
rc=$?; [ $rc -ge 124 ] && exit $rc
scripts/gpu_steps.sh \
  c4parts 300 "python -u scripts/c4_parts.py > gpurun_out/r6_c4_parts.txt" \
  shard_c2 300 "python -u scripts/shard_probe.py --config c2 --shards 1 2 4 8 --reps 2 > gpurun_out/r6_shard_probe_c2.txt" \
  shard_c4 400 "python -u scripts/shard_probe.py --config c4 --shards 1 8 --reps 2 > gpurun_out/r6_shard_probe_c4.txt"
