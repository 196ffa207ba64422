#!/bin/bash
# same-box F1 A/B: the round-3 tree (build/r3tree: git archive of the round-3 commit, its library built there)
# against this tree, interleaved twice
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
for r in 1 2; do
  for v in r3 r4; do
    if [ $v = r3 ]; then dir=build/r3tree; else dir=.; fi
    (cd $dir && timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline) > "$OUT/abr3_$v$r.log" 2>&1 || { tail -3 "$OUT/abr3_$v$r.log"; exit 1; }
    echo "$v $(tail -1 $OUT/abr3_$v$r.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"], d["roofline"]["mean_launch_ms"])')"
  done
done
exit 0
