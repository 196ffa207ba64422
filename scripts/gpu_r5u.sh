#!/bin/bash
# round 5: the channel-stationary BatchNorm apply kernels (es_set_bn_cs): bit-identity and Conformer / ResNet tests,
# then S1 A/B (same tree, interleaved)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_conformer.py tests/test_gpu_resnet.py tests/test_gpu_convs.py > "$OUT/tb.log" 2>&1; rc=$?; tail -2 "$OUT/tb.log"; [ $rc -ne 0 ] && exit 1
arm() {  # arm <name> <cs> <bench args...>
  local name=$1 b=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); from endossl import _lib; _lib.load().es_set_bn_cs($b); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm s1c0_$r 0 --workload s1 --steps 5 --warmup 2 || exit 1
  arm s1c1_$r 1 --workload s1 --steps 5 --warmup 2 || exit 1
done
exit 0
