#!/bin/bash
# round 4 confirm: the whole GPU suite, smoke(), the default bench line, then the step counters (TAG=r04)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-1200; return $rc; }
run suite 900 python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 420 python -u bench.py || exit 1
if [ -z "$NOCNT" ]; then bash scripts/gpu_step_counters.sh > "$OUT/cnt.log" 2>&1; echo "counters rc=$?"; tail -4 "$OUT/cnt.log"; fi
exit 0
