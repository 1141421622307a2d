#!/bin/bash
# Build a committed revision (default HEAD) into _ab_prev/ for same-box A/B runs against the working
# tree (scripts/ab_prev.sh). The worktree lives under /tmp; only the built library and the Python
# needed to run bench.py / shard_probe.py are copied in.
set -eo pipefail
rev=${1:-HEAD}
wt=/tmp/ab_prev_wt
root=$(git -C "$(dirname "$0")/.." rev-parse --show-toplevel)
[ -d $wt ] || git -C "$root" worktree add -f $wt "$rev" -q
git -C $wt checkout -q --detach "$(git -C "$root" rev-parse "$rev")"
rm -rf $wt/ray-tracing_amd/build  # (a stale library must never stand in for a failed build)
make -s -j8 -C $wt/ray-tracing_amd/csrc
rm -rf "$root/_ab_prev"; mkdir -p "$root/_ab_prev/tests/golden"
cp -r $wt/bench.py $wt/scripts $wt/ray-tracing_amd "$root/_ab_prev/"
cp $wt/tests/golden/earthmap_rgb8.npz "$root/_ab_prev/tests/golden/"
rm -f "$root"/_ab_prev/ray-tracing_amd/build/*.o
echo "_ab_prev = $(git -C $wt log --oneline -1)"
