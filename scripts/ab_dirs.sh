#!/bin/bash
# Same-box A/B of bench kernel times: the working tree against each given build directory
# (_ab_prev/ from scripts/ab_prev_build.sh, _var_*/ from build_variant.sh / build_patched.sh),
# alternating twice. usage: scripts/ab_dirs.sh "<bench args>" dir1 [dir2 ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
args=$1; shift
run() { timeout -k 10 ${AB_TIMEOUT:-300} python -u bench.py --no-cpu-baseline --no-work $args 2>&1 | grep -o 'kernel [0-9.]* ms' | tr '\n' ' '; echo; }
for rep in 1 2; do
  echo "tree: $(run)"
  for d in "$@"; do echo "$d: $(cd $d && run)"; done
done
