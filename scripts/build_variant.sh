#!/bin/bash
# Build the working tree with extra compiler flags into _var_<name>/ (bench.py, scripts and the
# package with its library), for same-box A/B runs of code-generation options.
# usage: scripts/build_variant.sh <name> "<extra hipcc flags>"
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
src=/tmp/var_src_$name
rm -rf "$src"; mkdir -p "$src"
cp -r "$root/ray-tracing_amd" "$root/include" "$src/"
rm -rf "$src/ray-tracing_amd/build"
make -s -C "$src/ray-tracing_amd/csrc" EXTRA="$flags" > "$src/build.log" 2>&1 || { tail -5 "$src/build.log"; exit 1; }
out="$root/_var_$name"
rm -rf "$out"; mkdir -p "$out/tests/golden"
cp -r "$root/bench.py" "$root/scripts" "$out/"
mkdir -p "$out/ray-tracing_amd/build"
cp -r "$src/ray-tracing_amd/rtamd" "$out/ray-tracing_amd/"
cp "$src/ray-tracing_amd/build/librtamd.so" "$out/ray-tracing_amd/build/"
cp "$root/tests/golden/earthmap_rgb8.npz" "$out/tests/golden/"
echo "_var_$name built with: $flags"
