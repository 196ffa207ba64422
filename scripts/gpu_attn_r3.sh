#!/bin/bash
# attention microbenchmark + SQ counter passes + HBM bytes (FETCH / WRITE) of the F1 attention kernels
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 120 python scripts/attn_bench.py --rounds 3 --iters 10 > "$OUT/attnb.log" 2>&1; echo "bench rc=$?"; tail -4 "$OUT/attnb.log"
bash scripts/gpu_pmc_attn3.sh || exit 1
B="python3 $GRAFT_REPO_ROOT/scripts/attn_bench.py --rounds 1 --iters 2"
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/attnhbm_$i" -o run --output-format csv -- $B > "$OUT/attnhbm_$i.log" 2>&1
  rc=$?; echo "hbm pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
