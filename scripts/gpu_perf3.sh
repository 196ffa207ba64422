#!/bin/bash
# Round-3 perf iteration: kernel tests for the changed kernels, micro-benches (attention backward pipelined vs
# plain, TN weight gradient asm-DMA vs builtin), then the F1 bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-6}; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread"
run kt 400 $PT -m gpu -x tests/test_gpu_kernels.py tests/test_gpu_step.py; rc=$?
ok $rc && { TAILN=3 run attn 200 python scripts/attn_bench.py --rounds 5 --iters 10; rc=$?; }
ok $rc && { TAILN=8 run tn 300 python scripts/gemm_bench.py --only fc1_wgrad,fc2_wgrad,qkv_wgrad,proj_wgrad --tn-variants 7,9 --tn-blocks auto,s16 --rounds 5; rc=$?; }
ok $rc && { TAILN=8 run tnsh 300 python scripts/gemm_bench.py --only fc1_wgrad,fc2_wgrad,qkv_wgrad,proj_wgrad --tn-variants 0 --tn-blocks auto --rounds 5 --shard 8; rc=$?; }
ok $rc && { TAILN=2 run bench 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline; rc=$?; }
exit 0
