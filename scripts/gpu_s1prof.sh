#!/bin/bash
# S1 (Conformer-B/384) bench line, then a kernel-trace profile of 2 timed steps -> summary (TAG, default r04_s1)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
TAG=${TAG:-r04_s1}
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400; return $rc; }
run s1bench 400 python -u bench.py --workload s1 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
rm -rf "$OUT/s1prof"
run s1prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/s1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload s1 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
exit 0
