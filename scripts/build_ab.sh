#!/bin/bash
# Build libendossl_hip.so from the csrc/ of a git ref into OUT (for same-box A/B runs via ENDOSSL_LIB):
#   scripts/build_ab.sh <git-ref> <out.so>
set -e
ref=$1; out=$(realpath -m "$2")
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d /tmp/ab_XXXX)
git -C "$root" archive "$ref" endoscopy-image-classification_amd/csrc | tar -x -C "$tmp"
make -C "$tmp/endoscopy-image-classification_amd/csrc" -j8 OUT="$out" "$out" > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
rm -rf "$tmp"
echo "built $out from $ref"
