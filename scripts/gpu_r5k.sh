#!/bin/bash
# round 5: BatchNorm num_batches_tracked folded into the statistics launches, the conv weights packed in one
# launch per step (conformer.CONV_PACK_MULTI): the conv / Conformer / ResNet / kernel tests, then same-box
# interleaved S1 and P0 A/Bs of the one-launch pack against the per-weight pack
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_convs.py tests/test_gpu_conformer.py tests/test_gpu_resnet.py > "$OUT/tk.log" 2>&1; rc=$?; tail -3 "$OUT/tk.log"; [ $rc -ne 0 ] && exit 1
arm() {  # arm <name> <multi 0/1> <bench args...>
  local name=$1 multi=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.conformer as c; c.CONV_PACK_MULTI=bool($multi); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm s1a$r 0 --workload s1 --steps 5 --warmup 2 || exit 1
  arm s1b$r 1 --workload s1 --steps 5 --warmup 2 || exit 1
  arm p0a$r 0 --workload p0 --steps 50 --warmup 10 || exit 1
  arm p0b$r 1 --workload p0 --steps 50 --warmup 10 || exit 1
done
exit 0
