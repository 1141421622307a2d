#!/bin/bash
# Same-box A/B over the bench configs: the working tree against _ab_prev/ (scripts/ab_prev_build.sh),
# alternating twice. usage: scripts/ab_configs.sh [configs...]   (default: c2 c3 c5 c4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
cfgs=("$@"); [ ${#cfgs[@]} -eq 0 ] && cfgs=(c2 c3 c5 c4)
args() { case $1 in c5) echo "--config c5 --spp 16";; c4) echo "--config c4 --spp 100";; *) echo "--config $1";; esac; }
run() { timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-work --steps 3 --warmup 1 $(args $1) 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' '; echo; }
for rep in 1 2; do
  for c in "${cfgs[@]}"; do
    echo "tree $c: $(run $c)"
    echo "prev $c: $(cd _ab_prev && run $c)"
  done
done
