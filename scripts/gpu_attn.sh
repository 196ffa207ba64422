#!/bin/bash
# attention kernels: tests, microbenchmark, F1 bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run ka 300 $PT -m gpu -x tests/test_gpu_kernels.py -k "attention"; rc=$?
ok $rc && { run ab 200 python scripts/attn_bench.py; rc=$?; }
ok $rc && { run f1 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline; rc=$?; }
ok $rc && [ -n "$S1" ] && { run s1 400 python bench.py --workload s1 --steps 3 --warmup 2; rc=$?; }
exit 0
