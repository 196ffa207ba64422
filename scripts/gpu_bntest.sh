#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conformer.py -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "bn" > "$OUT/bnt.log" 2>&1; echo "new rc=$?"; tail -5 "$OUT/bnt.log"
ENDOSSL_LIB=$GRAFT_REPO_ROOT/build/r3tree/endoscopy-image-classification_amd/endossl/lib/libendossl_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_conformer.py -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "test_bn2d_fwd_bwd" > "$OUT/bnt_r3.log" 2>&1; echo "r3 lib rc=$?"; tail -5 "$OUT/bnt_r3.log"
exit 0
