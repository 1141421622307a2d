#!/bin/bash
# Round profiles for the headline config (and optionally others): GPU tests, bench lines, rocprofv3
# kernel stats and PMC passes, all under gpurun_out/; copy the summaries into profiles/ afterwards.
# usage: scripts/gpu_round_profiles.sh <round tag, e.g. r2> [extra configs...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r2}; shift
steps=(bench_c2 240 "python -u bench.py --steps 5 > gpurun_out/${tag}_bench_c2.json"
       stats_c2 240 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stats_c2 -o c2 -- python3 $PWD/bench.py --steps 3 --no-cpu-baseline --no-work"
       pmc_c2 600 "scripts/pmc_passes.sh gpurun_out/pmc_c2 --config c2")
for c in "$@"; do
  steps+=(bench_$c 300 "python -u bench.py --config $c --steps 1 --warmup 0 > gpurun_out/${tag}_bench_$c.json"
          stats_$c 300 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stats_$c -o $c -- python3 $PWD/bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-work")
done
scripts/gpu_steps.sh "${steps[@]}"
