#!/bin/bash
# attention variants at T = 577 (bit-exact, S1 A/B), then the S1 and N=8-shard kernel profiles
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out; export TMPDIR=/tmp
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT -x tests/test_gpu_kernels.py -k "attention_bwd_pipelined" > gpurun_out/ka.log 2>&1; rc=$?
echo "attn variants rc=$rc"; tail -2 gpurun_out/ka.log
[ $rc -eq 0 ] || exit 0
for r in 1 2; do
  for lv in 1 0; do
    ENDOSSL_ATTN_BWD_LONG=$lv timeout -k 10 300 python bench.py --workload s1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/s1l_$lv.log 2>&1 || exit 0
    echo "s1 attn_long=$lv: $(grep '^{' gpurun_out/s1l_$lv.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_s1maps" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --workload s1 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/prof_s1maps.log 2>&1
echo "prof s1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_shard8" -o run --output-format csv -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --batch 8 --no-cpu-baseline > gpurun_out/prof_shard8.log 2>&1
echo "prof shard rc=$?"
