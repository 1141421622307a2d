#!/bin/bash
# Same-box A/B of one config across build directories (the tree '.', _ab_prev, _var_*), alternating;
# extra environment per leg as DIR:VAR=VAL. usage: scripts/ab_dirs3.sh "<bench args>" dir[:ENV=V] ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
args=$1; shift
run() { timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-work $args 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' '; echo; }
for rep in 1 2; do
  for leg in "$@"; do
    d=${leg%%:*}; e=""; [ "$leg" != "$d" ] && e=${leg#*:}
    echo "$leg: $(cd "$d" && env $e bash -c "$(declare -f run); args='$args'; run")"
  done
done
