#!/bin/bash
# Same-box A/B of _ab_prev/ against the working tree on C2 (N = 1 and per shard at N = 8), C3, C4
# at 100 spp and C5 at 16 spp.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
echo "== c2"; scripts/ab_prev.sh
echo "== c3"; scripts/ab_config.sh --config c3
echo "== c4 100 spp"; scripts/ab_config.sh --config c4 --spp 100
echo "== c5 16 spp"; scripts/ab_config.sh --config c5 --spp 16
