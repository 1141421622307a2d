#!/bin/bash
# Build the working tree with a source patch (a python script editing files under its argv[1] dir)
# into _var_<name>/, for same-box A/B timing of experiments that are not (yet) in the tree.
# usage: scripts/build_patched.sh <name> <patch.py> ["<extra hipcc flags>"]
set -eo pipefail
name=$1; patch=$2; flags=${3:-}
root=$(cd "$(dirname "$0")/.." && pwd)
src=/tmp/var_src_$name
rm -rf "$src"; mkdir -p "$src"
cp -r "$root/ray-tracing_amd" "$root/include" "$src/"
rm -rf "$src/ray-tracing_amd/build"
python3 "$patch" "$src"
make -s -j8 -C "$src/ray-tracing_amd/csrc" EXTRA="$flags" > "$src/build.log" 2>&1 || { tail -5 "$src/build.log"; exit 1; }
out="$root/_var_$name"
rm -rf "$out"; mkdir -p "$out/tests/golden"
cp -r "$root/bench.py" "$root/scripts" "$out/"
mkdir -p "$out/ray-tracing_amd/build"
cp -r "$src/ray-tracing_amd/rtamd" "$out/ray-tracing_amd/"
cp "$src/ray-tracing_amd/build/librtamd.so" "$out/ray-tracing_amd/build/"
cp "$root/tests/golden/earthmap_rgb8.npz" "$out/tests/golden/"
echo "_var_$name built with patch $patch $flags"
