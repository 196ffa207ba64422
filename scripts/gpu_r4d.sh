#!/bin/bash
# round 4: attention tests (bit-identity of every backward variant, T = 197 and 577), the attention
# microbenchmarks (F1 / S1 shapes), attention HBM bytes, the F1 bench line, then the step counters (TAG=r04)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-800; return $rc; }
run ab 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" || exit 1
run abs1 200 python -u scripts/attn_bench.py --s1 --rounds 3 --no-fwd --bwd 3 || exit 1
bash scripts/gpu_attn_hbm.sh || exit 1
run bench 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
if [ -z "$NOCNT" ]; then bash scripts/gpu_step_counters.sh || exit 1; fi
exit 0
