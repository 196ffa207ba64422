#!/bin/bash
# round 5: the changed parity tests (SemiFormer decidable-row loss check, the F1 step against the fp32 oracle,
# per-op parity at the N = 8 shard, the restored pruned-row / grouped-wgrad tests), then the default bench line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-400; return $rc; }
PT="python -u -m pytest -v -rf -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
run sf 300 $PT tests/test_gpu_conformer.py -k semiformer_trainer -s; rc1=$?
[ $rc1 -gt 1 ] && exit $rc1
run par 400 $PT tests/test_gpu_parity.py -k full_size -s; rc2=$?
[ $rc2 -gt 1 ] && exit $rc2
run blk 600 $PT tests/test_gpu_blocks.py -s; rc3=$?
[ $rc3 -gt 1 ] && exit $rc3
run stp 300 $PT tests/test_gpu_step.py -k "grouped or last_block"; rc4=$?
[ $rc4 -gt 1 ] && exit $rc4
run bench 400 python bench.py || exit 1
exit 0
