#!/bin/bash
# same-box A/B at the N = 8 per-rank shard (B = 8, mu = 7 on one GPU): knob sets in AV, interleaved twice
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for r in 1 2; do
  for v in ${AV:-es_set_attn_bwd_variant=3 es_set_attn_bwd_variant=4 es_set_attn_bwd_variant=4,es_set_attn_bwd_grid=384}; do
    i=$((i+1))
    timeout -k 10 240 python -u scripts/s1_knob_ab.py $(echo $v | tr "," " ") --batch ${SB:-8} --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/absh_$i.log" 2>&1 || { tail -3 "$OUT/absh_$i.log"; exit 1; }
    echo "$v $(tail -1 $OUT/absh_$i.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
  done
done
exit 0
