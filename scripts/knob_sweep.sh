#!/bin/bash
# A/B sweep of the render kernel's env knobs on one config: one bench line per setting.
# usage: [BENCH_ARGS="--spp 100"] scripts/knob_sweep.sh <config> "<ENV=.. ENV=..>" ["<ENV=..>" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
cfg=$1; shift
for setting in "$@"; do
  line=$(env $setting timeout -k 10 120 python bench.py --config "$cfg" --steps 3 --warmup 1 \
         --no-cpu-baseline --no-work $BENCH_ARGS 2>/dev/null) || { echo "FAIL [$setting] rc=$?"; exit 1; }
  ms=$(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')
  echo "$cfg [$setting] ms/value: $ms" | tee -a gpurun_out/sweep.log
done
