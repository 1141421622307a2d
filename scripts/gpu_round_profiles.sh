#!/bin/bash
# Round profiles: bench lines, rocprofv3 kernel stats and PMC passes, all under gpurun_out/; copy the
# summaries into profiles/ afterwards.
# usage: scripts/gpu_round_profiles.sh <round tag, e.g. r2> [c2|c3|c4|c5 ...]   (default: c2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r2}; shift
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=(c2)
steps=()
for c in "${cfgs[@]}"; do
  case $c in
    c2) b="--steps 5"; s="--steps 3";;
    c5) b="--config c5 --spp 16 --steps 3"; s="--config c5 --spp 16 --steps 2";;
    c1) b="--config c1 --steps 20 --warmup 3"; s="--config c1 --steps 20 --warmup 3";;  # (launch-bound: warm up)
    *)  b="--config $c --steps 1 --warmup 0"; s="--config $c --steps 1 --warmup 0";;
  esac
  steps+=(bench_$c 400 "python -u bench.py $b > gpurun_out/${tag}_bench_$c.json"
          stats_$c 300 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stats_$c -o $c -- python3 $PWD/bench.py $s --no-cpu-baseline --no-work")
  case $c in c2) steps+=(pmc_c2 600 "scripts/pmc_passes.sh gpurun_out/pmc_c2 --config c2");; c5) steps+=(pmc_c5 600 "scripts/pmc_passes.sh gpurun_out/pmc_c5 --config c5 --spp 16");; esac
done
scripts/gpu_steps.sh "${steps[@]}"
