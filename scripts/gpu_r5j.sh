#!/bin/bash
# round 5: S1 A/B of the N = 768 NT rule (A = the previous build, B = the tree), then a serialised S1 kernel
# profile (branch stream and side-stream weight gradients off: every kernel's isolated time)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
R=3 LIM=200 BARGS="--workload s1 --steps 5 --warmup 2" bash scripts/gpu_ab_lib.sh || exit 1
rm -rf "$OUT/s1ser"
ser="import sys; sys.argv=['bench.py','--workload','s1','--steps','2','--warmup','1','--no-cpu-baseline']; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.conformer as c; c.BRANCH_STREAMS=False; c.CONV_DW_SIDE=False; import runpy; runpy.run_path('bench.py', run_name='__main__')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/s1ser" -o run --output-format csv -- python3 -c "$ser" > "$OUT/s1ser.log" 2>&1; rc=$?; echo "s1 serial prof rc=$rc"; tail -1 "$OUT/s1ser.log" | cut -c1-200
exit $rc
