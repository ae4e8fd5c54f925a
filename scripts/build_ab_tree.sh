#!/bin/bash
# Build libsdrhip.so from the WORKING TREE's package sources with extra
# compiler flags into ab/<name>.so, for same-box A/B timing of build-time
# switches:   bash scripts/build_ab_tree.sh nt -DSDR_FIR_NT=1
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
PKG=3dy4-real-time-software-defined-radio-_amd
tmp=$(mktemp -d)
mkdir -p ab
objs=()
for f in "$PKG"/csrc/*.hip; do
  o="$tmp/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
    -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -I"$PKG/csrc" "$@" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/$name.so" "${objs[@]}"
rm -rf "$tmp"
echo "ab/$name.so"
