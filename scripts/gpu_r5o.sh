#!/bin/bash
# round 5: which BatchNorm -> conv pairs to fuse (conformer.BN_CONV_FUSED / BN_CONV_FUSED_KXK): S1 and P0,
# same box, interleaved arms A = every pair fused, B = 1 x 1 convs only, C = none
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
arm() {  # arm <name> <fused> <kxk> <bench args...>
  local name=$1 fu=$2 kk=$3; shift 3
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); import endossl.conformer as c; c.BN_CONV_FUSED=bool($fu); c.BN_CONV_FUSED_KXK=bool($kk); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm s1A$r 1 1 --workload s1 --steps 5 --warmup 2 || exit 1
  arm s1B$r 1 0 --workload s1 --steps 5 --warmup 2 || exit 1
  arm s1C$r 0 0 --workload s1 --steps 5 --warmup 2 || exit 1
done
for r in 1 2 3; do
  arm p0A$r 1 1 --workload p0 --steps 100 --warmup 10 || exit 1
  arm p0C$r 0 0 --workload p0 --steps 100 --warmup 10 || exit 1
done
exit 0
