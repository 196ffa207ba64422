#!/bin/bash
# A/B of Engine.RESID_LN (es_gemm_nt_resid_ln: the attention projection + residual + LayerNorm 2 in one launch) on
# one box, interleaved: F1 and the N = 8 shard, three runs each way; the isolated launch at every per-rank size first
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 150 python -u scripts/resid_ln_bench.py > "$OUT/rlb.log" 2>&1 || { tail -5 "$OUT/rlb.log"; exit 1; }
grep "{" "$OUT/rlb.log"
for i in 1 2 3; do
  for v in 0 1; do
    ENDOSSL_RESID_LN=$v timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline > "$OUT/rl_f1_${v}_$i.log" 2>&1 || { tail -5 "$OUT/rl_f1_${v}_$i.log"; exit 1; }
    echo "F1 resid_ln=$v run $i: $(tail -1 "$OUT/rl_f1_${v}_$i.log" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
exit 0
