#!/bin/bash
# stream priorities: N = 8 shard (B = 8) with the ViT side stream at -1 vs 0, then S1 branch / wgrad priorities
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
R=2 BARGS="--batch 8" AV="endossl.vit.SIDE_PRIORITY=0 endossl.vit.SIDE_PRIORITY=-1" bash scripts/gpu_ab_knobs3.sh || exit 1
echo S1
i=0
for r in 1 2; do
  for v in "endossl.conformer.BRANCH_PRIORITY=0" "endossl.conformer.WGRAD_PRIORITY=-1" "endossl.conformer.BRANCH_PRIORITY=-1" "endossl.conformer.BRANCH_PRIORITY=-1,endossl.conformer.WGRAD_PRIORITY=-1"; do
    i=$((i+1))
    timeout -k 10 300 python -u scripts/s1_knob_ab.py $(echo $v | tr "," " ") > "$OUT/abs_$i.log" 2>&1 || { tail -3 "$OUT/abs_$i.log"; exit 1; }
    echo "$v $(tail -1 $OUT/abs_$i.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
  done
done
