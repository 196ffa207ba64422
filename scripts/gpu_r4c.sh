#!/bin/bash
# round 4: attention backward variants (bit-identity) + attention microbenchmark
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-600; return $rc; }
run ab 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention_bwd" || exit 1
run abench 300 python -u scripts/attn_bench.py --rounds 3 || exit 1
exit 0
