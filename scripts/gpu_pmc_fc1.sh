#!/bin/bash
# HBM traffic of the bench's roofline kernel (train fc1 forward, default NT variant): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes (no tracing), over scripts/gemm_bench.py.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/scripts/gemm_bench.py --variants=-1 --rounds 1 --iters 2 --only fc1_fwd --tn-blocks 1536"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/fc1pmc$i" -o run --output-format csv -- $B > "$OUT/fc1pmc$i.log" 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/fc1pmc$i.log"; exit $rc; }
done
exit 0
