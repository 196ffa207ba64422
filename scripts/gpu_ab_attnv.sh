#!/bin/bash
# same-box F1 A/B of the attention backward: knob sets in AV (space-separated; within a set, comma-separated
# es_set_...=v), interleaved twice.  Default: two-pass (variant 3) vs the single pass on all CUs vs on 160
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for r in 1 2; do
  for v in ${AV:-es_set_attn_bwd_variant=3 es_set_attn_bwd_variant=4 es_set_attn_bwd_variant=4,es_set_attn_bwd_grid=160}; do
    i=$((i+1))
    timeout -k 10 240 python -u scripts/s1_knob_ab.py $(echo $v | tr "," " ") --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/abav_$i.log" 2>&1 || { tail -3 "$OUT/abav_$i.log"; exit 1; }
    echo "$v $(tail -1 $OUT/abav_$i.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"], d["roofline"]["mean_launch_ms"])')"
  done
done
exit 0
