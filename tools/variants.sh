#!/bin/bash
# Build measurement-only variants of the product kernel into tools/variants/ (never shipped):
#   tools/variants.sh NAME "-DFLAG ..." [NAME "-D..." ...]
# Select one at run time with NSTACK_FCS_LIB=tools/variants/libfcs_NAME.so.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
mkdir -p "$HERE/variants"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  # each build in its own directory: concurrent hipcc runs in one directory clobber each other's
  # offload intermediates (a variant then silently went missing)
  ( d=$(mktemp -d) && cd "$d" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags \
     -o "$HERE/variants/libfcs_$name.so" "$ROOT/nstack_amd/csrc/fcs_kernel.hip" "$ROOT/nstack_amd/csrc/inet_kernel.hip" \
     "$ROOT"/nstack_amd/csrc/*.cpp -lpthread > "$d/log" 2>&1 || { echo "variant $name failed:"; tail -5 "$d/log"; }
    rm -rf "$d" ) &
done
wait
ls "$HERE/variants"
