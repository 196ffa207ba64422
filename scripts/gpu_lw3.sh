#!/bin/bash
# grouped block weight gradients: kernel + step/block tests, F1 CU-share sweep, C1 / shard / S1 A/Bs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
run kt 300 $PT -m gpu tests/test_gpu_kernels.py -k tn || exit 1
run ts 400 $PT -m gpu tests/test_gpu_step.py tests/test_gpu_blocks.py tests/test_gpu_parity.py -x || exit 1
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
for r in 1 2; do
  for sh in 0.25 0.3125 0.375 0.4375 0.5; do ENDOSSL_LAYER_TN_SHARE=$sh run sh_${sh}_$r 200 $B || exit 1; done
done
ENDOSSL_LAYER_WGRAD=0 run f1_off 200 $B || exit 1
for sh in 0.375 0.5; do ENDOSSL_LAYER_TN_SHARE=$sh run c1_$sh 300 python bench.py --workload c1 --steps 5 --warmup 2 || exit 1; done
ENDOSSL_LAYER_WGRAD=0 run c1_off 300 python bench.py --workload c1 --steps 5 --warmup 2 || exit 1
for sh in 0.375 0.5; do ENDOSSL_LAYER_TN_SHARE=$sh run shard2_$sh 200 $B --batch 32 || exit 1; done
ENDOSSL_LAYER_WGRAD=0 run shard2_off 200 $B --batch 32 || exit 1
for sh in 0.5 0.75; do ENDOSSL_CONF_TN_SHARE=$sh run s1_$sh 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1; done
ENDOSSL_LAYER_WGRAD=0 run s1_off 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
exit 0
