#!/bin/bash
# Round-end evidence in one GPU call (everything under gpurun_out/; copy what is judged into profiles/):
# the GPU test suite, rocprofv3 kernel stats + PMC passes + the bench line of every config
# (scripts/gpu_round_profiles.sh), and the per-shard probes of C2, C4 and C5 at 1 and 8 shards.
# usage: scripts/gpu_round_final.sh <round tag, e.g. r4> [configs...]   (default: c1 c2 c3 c4 c5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r4}; shift
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=(c1 c2 c3 c4 c5)
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }  # (a test failure is not: go on)
scripts/gpu_steps.sh gputest 900 "python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread"
rc=$?; fatal $rc && exit $rc
scripts/gpu_round_profiles.sh "$tag" "${cfgs[@]}"
rc=$?; fatal $rc && exit $rc
scripts/gpu_steps.sh \
  shard_c2 300 "python -u scripts/shard_probe.py --config c2 --shards 1 2 4 8 --reps 2 > gpurun_out/${tag}_shard_probe_c2.txt" \
  shard_c4 400 "python -u scripts/shard_probe.py --config c4 --shards 1 8 --reps 2 > gpurun_out/${tag}_shard_probe_c4.txt" \
  shard_c5 600 "python -u scripts/shard_probe.py --config c5 --shards 1 8 --reps 1 > gpurun_out/${tag}_shard_probe_c5.txt"
