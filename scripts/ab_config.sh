#!/bin/bash
# Same-box A/B of one config's bench line: _ab_prev/ (scripts/ab_prev_build.sh) vs the working tree,
# alternating. usage: scripts/ab_config.sh <bench args...>   e.g. --config c4 --spp 100
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
run() { timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work "$@" 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' '; echo; }
for i in 1 2; do
  echo "prev: $(cd _ab_prev && run "$@")"
  echo "new:  $(run "$@")"
done
