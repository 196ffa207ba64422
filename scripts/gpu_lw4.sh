#!/bin/bash
# the grouped block weight gradients at the default share: conformer opt-in test, F1 bench, PMC passes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread"
ENDOSSL_CONF_LAYER_WGRAD=1 run tc 400 $PT -m gpu tests/test_gpu_conformer.py -x || exit 1
run f1 200 python bench.py --steps 10 --warmup 3 || exit 1
bash scripts/gpu_pmc_step.sh
exit 0
