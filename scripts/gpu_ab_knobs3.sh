#!/bin/bash
# scripts/gpu_ab_knobs.sh with R rounds (default 3)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for r in $(seq ${R:-3}); do
  for v in $AV; do
    i=$((i+1))
    timeout -k 10 240 python -u scripts/s1_knob_ab.py $(echo $v | tr "," " ") --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BARGS} > "$OUT/abk_$i.log" 2>&1 || { tail -3 "$OUT/abk_$i.log"; exit 1; }
    echo "$v $(tail -1 $OUT/abk_$i.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"])')"
  done
done
exit 0
