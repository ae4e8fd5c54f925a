#!/bin/bash
# Build libsdrhip.so from the package sources at git revision $1 into
# ab/<name>.so ($2, default = the revision), for same-box A/B timing:
#   SDRHIP_LIB=ab/<name>.so python bench.py ...
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=${2:-$1}
PKG=3dy4-real-time-software-defined-radio-_amd
tmp=$(mktemp -d)
git archive "$rev" "$PKG/csrc" include | tar -x -C "$tmp"
mkdir -p ab
objs=()
for f in "$tmp/$PKG"/csrc/*.hip; do
  o="$tmp/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize \
    -fhip-fp32-correctly-rounded-divide-sqrt -I"$tmp/include" -I"$tmp/$PKG/csrc" -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "ab/$name.so" "${objs[@]}"
rm -rf "$tmp"
echo "ab/$name.so"
