#!/bin/bash
# round 5: the bf16 convs with the BatchNorm applied by the gather (es_conv2d_*_bf16_bnin_ex) against the plain
# gather, per ConvBlock shape (scripts/convb_bench.py --bnin), for the previous build (A) and the tree's (B)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
A=$PWD/endoscopy-image-classification_amd/csrc/build/ab/libA.so
for r in 1 2; do
  ENDOSSL_LIB=$A timeout -k 10 200 python3 scripts/convb_bench.py --bnin --iters 7 > "$OUT/cbA$r.log" 2>&1 || { tail -3 "$OUT/cbA$r.log"; exit 1; }
  timeout -k 10 200 python3 scripts/convb_bench.py --bnin --iters 7 > "$OUT/cbB$r.log" 2>&1 || { tail -3 "$OUT/cbB$r.log"; exit 1; }
done
for f in cbA1 cbB1 cbA2 cbB2; do echo "== $f"; grep -v "^/opt\|amdgpu.ids" "$OUT/$f.log"; done
exit 0
