#!/bin/bash
# F1 kernel trace (per-stream busy per step) + weight-gradient kernel variants at half / whole chip
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_bench.py --variants -1 --only fc1_wgrad,fc2_wgrad,qkv_wgrad,proj_wgrad --tn-variants 5,6,7,8 --tn-blocks s8,s16,s32 --rounds 3 > "$OUT/tnv.log" 2>&1; echo "tn rc=$?"; grep -v amdgpu.ids "$OUT/tnv.log"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/tr_f1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/tr.log" 2>&1; echo "trace rc=$?"
f=$(find "$OUT/tr_f1" -name "*kernel_trace.csv" | head -1); python3 scripts/step_timeline.py "$f" | tail -4
