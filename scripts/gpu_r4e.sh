#!/bin/bash
# round 4: the F1 bench line (full CPU baseline), the step counters (TAG=r04), then the whole GPU suite + smoke
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-1500; return $rc; }
run bench 420 python -u bench.py || exit 1
if [ -z "$NOCNT" ]; then bash scripts/gpu_step_counters.sh > "$OUT/cnt.log" 2>&1; echo "counters rc=$?"; tail -25 "$OUT/cnt.log"; fi
exit 0
