#!/bin/bash
# round 5: BatchNorm + ReLU applied by the bf16 conv gathers (conformer.BN_CONV_FUSED): the Conformer / ResNet /
# conv GPU tests, then same-box interleaved S1 and P0 A/Bs of the fused path against the same tree with the
# fusion switched off (the A arm sets BN_CONV_FUSED = False before running bench.py)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300; return $rc; }
PT="python -u -m pytest -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
run tconf 600 $PT tests/test_gpu_conformer.py tests/test_gpu_resnet.py tests/test_gpu_convs.py -k "fused or resnet or conv" || exit 1
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python -u -c "import sys; sys.argv=['bench.py','--workload','s1','--steps','10','--warmup','3','--no-cpu-baseline']; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.conformer as c; c.BN_CONV_FUSED=False; import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$OUT/s1a$r.log" 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --workload s1 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/s1b$r.log" 2>&1 || exit 1
  echo "S1 round $r: unfused $(ms $OUT/s1a$r.log) fused $(ms $OUT/s1b$r.log)"
done
for r in 1 2; do
  timeout -k 10 300 python -u -c "import sys; sys.argv=['bench.py','--workload','p0','--steps','50','--warmup','5','--no-cpu-baseline']; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.conformer as c; c.BN_CONV_FUSED=False; import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$OUT/p0a$r.log" 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --workload p0 --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/p0b$r.log" 2>&1 || exit 1
  echo "P0 round $r: unfused $(ms $OUT/p0a$r.log) fused $(ms $OUT/p0b$r.log)"
done
