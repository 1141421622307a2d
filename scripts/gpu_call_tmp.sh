# round-6 evidence, part 2: C1, C3, C4 profiles (rocprofv3 stats, PMC passes) and bench lines
cd "${GRAFT_REPO_ROOT:-.}" || exit 2
scripts/gpu_round_profiles.sh r6 c4 c3 c1
