#!/bin/bash
# GPU pass: kernel tests, step tests, smoke, bench, rocprofv3 kernel trace of the bench.
# Each GPU step has its own time limit; a crash/timeout (rc > 1) stops the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -3 "$OUT/$name.log"
  return $rc
}
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run t 1100 $PT -m gpu -x tests/; rc=$?   # the driver's round-end GPU tier: every gpu test, one process
ok $rc && { run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; }
ok $rc && { run bench 600 python bench.py --steps 10 --warmup 3; rc=$?; }
ok $rc && { run c1 300 python bench.py --workload c1 --steps 5 --warmup 2; rc=$?; }
ok $rc && { run s1 400 python bench.py --workload s1 --steps 3 --warmup 2; rc=$?; }
ok $rc && { run p0 200 python bench.py --workload p0 --steps 10 --warmup 3; rc=$?; }
if ok $rc && [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline; rc=$?
fi
exit 0
