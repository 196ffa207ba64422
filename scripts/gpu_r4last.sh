#!/bin/bash
# last round-4 check: embedding-backward kernel (test + timing vs the per-feature kernel), the whole GPU suite,
# smoke(), the default bench line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
for p in 0 1 0 1; do timeout -k 10 120 python scripts/embed_bench.py --pad $p 2>&1 | grep embed_bwd || exit 1; done
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300; return $rc; }
run suite 900 python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run bench 420 python -u bench.py || exit 1
exit 0
