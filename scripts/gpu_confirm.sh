#!/bin/bash
# what the driver runs at round end: the GPU suite, smoke(), the default bench line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300; return $rc; }
run t 900 python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu -x tests/ || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 400 python bench.py || exit 1
exit 0
