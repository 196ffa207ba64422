#!/bin/bash
# round 5: LayerNorm parameter gradients deferred off the data-gradient chain (Engine.DEFER_LN_GRADS): the step
# tests, then F1 and N = 8 shard A/Bs against the tree with the deferral off (interleaved, same box)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_blocks.py tests/test_gpu_parity.py tests/test_gpu_kernels.py -k "deferred or layernorm or ln_ or grouped or lanes or f1 or full_size" > "$OUT/tp.log" 2>&1; rc=$?; tail -3 "$OUT/tp.log"; [ $rc -ne 0 ] && exit 1
arm() {  # arm <name> <defer 0/1> <bench args...>
  local name=$1 d=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.vit as v; v.Engine.DEFER_LN_GRADS=bool($d); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm f1A$r 0 --steps 100 --warmup 5 || exit 1
  arm f1B$r 1 --steps 100 --warmup 5 || exit 1
  arm shA$r 0 --batch 8 --steps 200 --warmup 10 || exit 1
  arm shB$r 1 --batch 8 --steps 200 --warmup 10 || exit 1
done
exit 0
