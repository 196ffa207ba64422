#!/bin/bash
# deterministic head weight gradient: kernel test, the step tests, and two bench runs whose final losses must match
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_comatch.py -k "cls_head or step or comatch" > "$OUT/thd.log" 2>&1; rc=$?; tail -2 "$OUT/thd.log"; [ $rc -ne 0 ] && exit 1
for k in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bd$k.log" 2>&1 || exit 1; tail -1 "$OUT/bd$k.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["final_loss"])'; done
