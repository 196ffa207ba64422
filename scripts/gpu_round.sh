#!/bin/bash
# GPU tests + an F1 A/B pair (ABV) + S1 with the host input path
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log"; return $rc; }
ok() { [ "$1" -le 1 ]; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run t 1100 $PT -m gpu -x tests/; rc=$?
ok $rc && [ -n "$ABV" ] && { bash scripts/gpu_ab_f1.sh; rc=$?; }
ok $rc && { run s1h 500 python bench.py --workload s1 --steps 3 --warmup 2 --host-input; rc=$?; }
exit 0
