#!/bin/bash
# Build the library of a git revision (default HEAD) into build/ab/<rev>/libendossl_hip.so, for same-box
# A/B runs with ENDOSSL_LIB=<that path>.  usage: bash scripts/build_ab_lib.sh [rev]
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D="$ROOT/build/ab/$REV"
rm -rf "$D/src" && mkdir -p "$D/src"
git -C "$ROOT" archive "$REV" endoscopy-image-classification_amd/csrc | tar -x -C "$D/src"
make -C "$D/src/endoscopy-image-classification_amd/csrc" -j8 OUT="$D/libendossl_hip.so" > /dev/null
ls -la "$D/libendossl_hip.so"
