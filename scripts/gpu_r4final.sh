#!/bin/bash
# round-4 final confirm: GPU suite, smoke(), F1 bench line (default), S1 and N = 8 shard lines, step counters
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400; return $rc; }
run suite 900 python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 420 python -u bench.py || exit 1
run s1 400 python -u bench.py --workload s1 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
run shard 300 python -u bench.py --batch 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
bash scripts/gpu_step_counters.sh > "$OUT/cnt.log" 2>&1; echo "counters rc=$?"; tail -2 "$OUT/cnt.log"
exit 0
