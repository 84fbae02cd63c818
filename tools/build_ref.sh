#!/bin/bash
# Build the HIP library of another commit as an A/B variant (for tools/ab_bench.sh):
#   tools/build_ref.sh <commit> <name>  ->  <pkg>/build/<name>/libseg_hip.so
set -e
commit=$1; name=$2
pkg=iv2019-boosting-semantic-segmentation-with-weak-labels_amd
tmp=$(mktemp -d)
git archive "$commit" $pkg/csrc include | tar -x -C "$tmp"
make -C "$tmp/$pkg/csrc" -j8 > /dev/null
mkdir -p $pkg/build/$name
cp "$tmp/$pkg/libseg_hip.so" $pkg/build/$name/libseg_hip.so
rm -rf "$tmp"
echo "$pkg/build/$name/libseg_hip.so"
