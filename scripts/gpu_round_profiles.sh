#!/bin/bash
# Round profiles, per config: rocprofv3 kernel stats, PMC passes at the config's default launch
# (summarised by scripts/pmc_summary.py into profiles/<tag>_pmc_<c>.json on the box and into gpurun_out/),
# then the bench line, which cites that summary (roofline.traffic, valu_roofline). Everything lands
# under gpurun_out/; copy the summaries into profiles/ afterwards.
# usage: scripts/gpu_round_profiles.sh <round tag, e.g. r3> [c1|c2|c3|c4|c5 ...]   (default: c2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tag=${1:-r3}; shift
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=(c2)
steps=()
for c in "${cfgs[@]}"; do
  case $c in
    c2) b="--steps 20 --warmup 5"; s="--steps 3";;   # (the driver's bench command)
    c1) b="--config c1 --steps 20 --warmup 3"; s="--config c1 --steps 20 --warmup 3";;  # (launch-bound: warm up)
    c5) b="--config c5 --steps 1 --warmup 1"; s="--config c5 --steps 1 --warmup 0";;
    *)  b="--config $c --steps 2 --warmup 1"; s="--config $c --steps 1 --warmup 0";;
  esac
  steps+=(stats_$c 300 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stats_$c -o $c -- python3 $PWD/bench.py $s --no-cpu-baseline --no-work"
          pmc_$c 900 "scripts/pmc_passes.sh gpurun_out/pmc_$c --config $c && python scripts/pmc_summary.py gpurun_out/pmc_$c profiles/${tag}_pmc_$c.json && cp profiles/${tag}_pmc_$c.json gpurun_out/"
          bench_$c 600 "python -u bench.py $b > gpurun_out/${tag}_bench_$c.json")
done
scripts/gpu_steps.sh "${steps[@]}"
