#!/bin/bash
# End-of-round GPU pass: tests, smoke, F1 bench (+host input; and the default invocation), C1,
# S1, P0, rocprofv3 F1 summary
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run t 1100 $PT -m gpu -x tests/; rc=$?
ok $rc && { run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; }
ok $rc && { run bench 600 python bench.py --steps 10 --warmup 3 --host-input; rc=$?; }
ok $rc && { run bench1 300 python bench.py; rc=$?; }
ok $rc && { run c1b 300 python bench.py --workload c1 --steps 5 --warmup 2; rc=$?; }
ok $rc && { run s1 400 python bench.py --workload s1 --steps 3 --warmup 2; rc=$?; }
ok $rc && { run p0 200 python bench.py --workload p0 --steps 10 --warmup 3; rc=$?; }
if ok $rc; then
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline; rc=$?
fi
exit 0
