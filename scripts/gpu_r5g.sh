#!/bin/bash
# round 5: the Conformer blocks' grouped weight gradients (conformer.CONF_TN_GROUPED): tests, then S1 A/B
# (same tree, interleaved): per-Linear launches / grouped at CONF_TN_SHARE 0.5 / grouped at 0.375
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conformer.py -k "grouped or vit_b_384 or semiformer_trainer or side_stream" > "$OUT/tg.log" 2>&1; rc=$?; tail -2 "$OUT/tg.log"; [ $rc -ne 0 ] && exit 1
arm() {  # arm <name> <grouped> <share>
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline','--workload','s1','--steps','5','--warmup','2']; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.conformer as c; c.CONF_TN_GROUPED=bool($2); c.CONF_TN_SHARE=$3; import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$OUT/$1.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$1.log') if l.startswith('{\"metric')][-1]); print('$1', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm g0_$r 0 0.5 || exit 1
  arm g1_$r 1 0.5 || exit 1
  arm g2_$r 1 0.375 || exit 1
done
