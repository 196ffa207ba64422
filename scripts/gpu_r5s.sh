#!/bin/bash
# round 5: the ResNet-18 (P0) conv shapes with the staged kernels' branch-free loads off / on (convb_bench.py --bnin --p0)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
for b in 0 1 0 1; do timeout -k 10 200 python3 scripts/convb_bench.py --bnin --p0 --f32maps --iters 9 --dwbuf $b > "$OUT/p0c$b.log" 2>&1 || exit 1; echo "== dwbuf $b"; grep -v "^/opt\|amdgpu.ids" "$OUT/p0c$b.log" | cut -c1-200; done
