#!/bin/bash
# round 5: the bf16 convs on the LDS-DMA ring kernel (es_set_conv_ring: data gradients and non-widening forwards)
# and the division-free dense epilogue: ring bit-identity and conv / Conformer / ResNet tests, then S1 and P0 A/Bs
# of ring 0 vs 3 (same tree, interleaved)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_convs.py tests/test_gpu_conformer.py tests/test_gpu_resnet.py -k "conv or Conformer or conformer or resnet or semiformer or bn" > "$OUT/tc.log" 2>&1; rc=$?; tail -2 "$OUT/tc.log"; [ $rc -ne 0 ] && exit 1
arm() {  # arm <name> <ring> <bench args...>
  local name=$1 rg=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); from endossl import _lib; _lib.load().es_set_conv_ring($rg); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm s1r0_$r 0 --workload s1 --steps 5 --warmup 2 || exit 1
  arm s1r3_$r 3 --workload s1 --steps 5 --warmup 2 || exit 1
  arm p0r0_$r 0 --workload p0 --steps 200 --warmup 20 || exit 1
  arm p0r3_$r 3 --workload p0 --steps 200 --warmup 20 || exit 1
done
exit 0
