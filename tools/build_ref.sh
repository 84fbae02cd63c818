#!/bin/bash
# Build the HIP library of another commit as an A/B variant (for tools/ab_bench.sh):
#   tools/build_ref.sh <commit> <name>  ->  ab/<name>/libseg_hip.so (A/B only: delete after use)
set -e
commit=$1; name=$2
pkg=iv2019-boosting-semantic-segmentation-with-weak-labels_amd
tmp=$(mktemp -d)
git archive "$commit" $pkg/csrc include | tar -x -C "$tmp"
make -C "$tmp/$pkg/csrc" -j8 > /dev/null
mkdir -p ab/$name
cp "$tmp/$pkg/libseg_hip.so" ab/$name/libseg_hip.so
rm -rf "$tmp"
echo "ab/$name/libseg_hip.so"
