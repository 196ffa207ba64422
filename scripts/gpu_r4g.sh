#!/bin/bash
# round 4: S1 tests (per-op parity, conformer kernels, full-size step), then S1 bench lines, A/B of the new MLP
# epilogues is not switchable: compare against the previous measurements (141.6-142.0 ms)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-600; return $rc; }
run ts1 500 python -u -m pytest tests/test_gpu_s1_blocks.py tests/test_gpu_conformer.py -x -q -rf -s -p no:cacheprovider --timeout 300 --timeout-method thread || exit 1
for r in 1 2; do
  run s1b$r 300 python -u bench.py --workload s1 --steps 3 --warmup 2 --no-cpu-baseline || exit 1
done
exit 0
