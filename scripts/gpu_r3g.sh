#!/bin/bash
# Full GPU suite + smoke + F1 / C1 / S1 / P0 bench lines + F1 rocprof summary
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread"
run t 1000 $PT -m gpu tests/; rc=$?
ok $rc && { run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; }
ok $rc && { run bench 400 python bench.py --steps 20 --warmup 5; rc=$?; }
ok $rc && { run c1 300 python bench.py --workload c1 --steps 5 --warmup 2 --no-cpu-baseline; rc=$?; }
ok $rc && { run s1 400 python bench.py --workload s1 --steps 5 --warmup 2 --no-cpu-baseline; rc=$?; }
ok $rc && { run p0 200 python bench.py --workload p0 --steps 10 --warmup 3 --no-cpu-baseline; rc=$?; }
if ok $rc; then
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_f1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline; rc=$?
fi
exit 0
