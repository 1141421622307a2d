#!/bin/bash
# Same-box comparison of code-generation variants (scripts/build_variant.sh) against the working
# tree: C2 kernel time at N = 1 (scripts/shard_probe.py), then C5 at 16 spp and C4 at 100 spp.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
probe() { timeout -k 10 100 python scripts/shard_probe.py --shards 1 --reps 3 2>/dev/null | grep "N=" | sed 's/, ideal.*//'; }
run() { timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work "$@" 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' '; echo; }
for rep in 1 2; do
  echo "base c2: $(probe)"
  for d in _var_*; do echo "$d c2: $(cd $d && probe)"; done
done
echo "base c5: $(run --config c5 --spp 16)"
for d in _var_*; do echo "$d c5: $(cd $d && run --config c5 --spp 16)"; done
echo "base c4: $(run --config c4 --spp 100)"
for d in _var_*; do echo "$d c4: $(cd $d && run --config c4 --spp 100)"; done
