#!/bin/bash
# A/B of env settings on one config with the counting build's work per sample: one line per setting.
# usage: [BENCH_ARGS=".."] scripts/ab_work.sh <config> "<ENV=.. ENV=..>" ["<ENV=..>" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
cfg=$1; shift
for setting in "$@"; do
  line=$(env $setting timeout -k 10 180 python bench.py --config "$cfg" --steps 3 --warmup 1 \
         --no-cpu-baseline $BENCH_ARGS 2>/dev/null) || { echo "FAIL [$setting] rc=$?"; exit 1; }
  echo "$line" | python -c '
import json, sys
d = json.loads(sys.stdin.read())
w = d.get("work_per_sample", {})
print(sys.argv[1], "[" + sys.argv[2] + "]", "ms", d["ms_per_step"], "value", d["value"],
      "wide", w.get("wide_nodes"), "leaf", w.get("prim_tests"), "box", w.get("box_tests"),
      "util", d.get("lane_utilisation"))' "$cfg" "$setting" | tee -a gpurun_out/ab.log
done
