#!/bin/bash
# Build a measurement library from another copy of the sources (e.g. a git revision), for A/B runs
# against the working tree with tools/ab.py (never shipped):
#   tools/variant_from_tree.sh NAME REV [FLAGS]   -> tools/variants/libfcs_NAME.so built from `git show REV:...`
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
name=$1; rev=$2; flags=${3:-}
tmp=$(mktemp -d)
mkdir -p "$tmp/nstack_amd/csrc" "$tmp/include" "$HERE/variants"
for f in $(git -C "$ROOT" ls-tree --name-only "$rev" nstack_amd/csrc/ include/); do
  git -C "$ROOT" show "$rev:$f" > "$tmp/$f"
done
cd "$tmp/nstack_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags \
   -o "$HERE/variants/libfcs_$name.so" fcs_kernel.hip inet_kernel.hip *.cpp -lpthread
rm -rf "$tmp"
ls -la "$HERE/variants/libfcs_$name.so"
