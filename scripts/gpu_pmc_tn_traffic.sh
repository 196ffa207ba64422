#!/bin/bash
# HBM traffic of one es_gemm_tn call at the bench's roofline site (fc1 weight gradient, M = 100,864, the
# library's default kernel and split-K: gemm_tn_big_kernel + splitk_reduce + the bias partial reduction):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes (no tracing) over scripts/gemm_bench.py.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants 5 --rounds 1 --iters 2 --only fc1_wgrad --tn-variants=-1 --tn-blocks auto"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/tnpmc$i" -o run --output-format csv -- $B > "$OUT/tnpmc$i.log" 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/tnpmc$i.log"; exit $rc; }
done
exit 0
