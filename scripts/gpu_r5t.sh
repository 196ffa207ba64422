#!/bin/bash
# round 5: P0 A/B of the staged conv kernels' branch-free loads (es_set_conv_dw_buf 0 / 1), both orders, 4 rounds
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
arm() {  # arm <name> <dwbuf> <bench args...>
  local name=$1 b=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); from endossl import _lib; _lib.load().es_set_conv_dw_buf($b); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2; do
  arm p0b0_$r 0 --workload p0 --steps 300 --warmup 30 || exit 1
  arm p0b1_$r 1 --workload p0 --steps 300 --warmup 30 || exit 1
  arm p0c1_$r 1 --workload p0 --steps 300 --warmup 30 || exit 1
  arm p0c0_$r 0 --workload p0 --steps 300 --warmup 30 || exit 1
done
exit 0
