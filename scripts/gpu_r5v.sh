#!/bin/bash
# round 5: S1 with HEAD's library (A), HEAD + the two-iteration BatchNorm cs kernels (U), HEAD + the 16-byte
# channel sums (V): same box, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
AB="$GRAFT_REPO_ROOT/endoscopy-image-classification_amd/csrc/build/ab"
LIBS="A=$AB/libA.so U=$AB/libU.so V=$AB/libV.so" R=3 LIM=240 BARGS="--workload s1 --steps 5 --warmup 2" bash scripts/gpu_ab_lib.sh
