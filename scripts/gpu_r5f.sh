#!/bin/bash
# round 5: S1 A/B (A = HEAD, B = fc2 dgrad MULAUX at K >= 768 on the two-workgroup 256 x 128 tile) and
# F1 A/B/C (B; C = fc1 GELU epilogues on the 128 x 128 BK32 3-stage tile; D = proj forward on it, plain stores)
cd "$GRAFT_REPO_ROOT"; L=$PWD/endoscopy-image-classification_amd/csrc/build/ab
LIBS="A=$L/libA.so B=$L/libB.so" R=2 BARGS="--workload s1 --steps 10 --warmup 3" bash scripts/gpu_ab_lib.sh || exit 1
LIBS="B=$L/libB.so C=$L/libC.so D=$L/libD.so" R=2 BARGS="--steps 100 --warmup 5" bash scripts/gpu_ab_lib.sh || exit 1
