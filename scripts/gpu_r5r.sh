#!/bin/bash
# round 5: the conv weight gradient with branch-free loads / pixel walk (es_set_conv_dw_buf): bit-identity tests,
# per-shape timing with the knob at 0 / 1 (scripts/convb_bench.py --bnin --all-shapes), S1 and P0 A/Bs
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "conv_dw_branch_free or conv_ring" > "$OUT/tw.log" 2>&1; rc=$?; tail -2 "$OUT/tw.log"; [ $rc -ne 0 ] && exit 1
for b in 0 1; do  # (dw_buf also switches the staged forward / data-grad gathers)
  timeout -k 10 300 python3 scripts/convb_bench.py --bnin --all-shapes --iters 7 --dwbuf $b > "$OUT/cw$b.log" 2>&1 || { tail -3 "$OUT/cw$b.log"; exit 1; }
done
for f in cw0 cw1; do echo "== $f"; grep -v "^/opt\|amdgpu.ids" "$OUT/$f.log" | cut -c1-200; done
arm() {  # arm <name> <dwbuf> <bench args...>
  local name=$1 b=$2; shift 2
  timeout -k 10 240 python3 -c "import sys; sys.argv=['bench.py','--no-cpu-baseline']+sys.argv[1:]; sys.path.insert(0,'endoscopy-image-classification_amd'); from endossl import _lib; _lib.load().es_set_conv_dw_buf($b); import runpy; runpy.run_path('bench.py', run_name='__main__')" "$@" > "$OUT/$name.log" 2>&1 || return 1
  python3 -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{\"metric')][-1]); print('$name', d['ms_per_step'])"
}
for r in 1 2 3; do
  arm s1b0_$r 0 --workload s1 --steps 5 --warmup 2 || exit 1
  arm s1b1_$r 1 --workload s1 --steps 5 --warmup 2 || exit 1
done
for r in 1 2; do
  arm p0b0_$r 0 --workload p0 --steps 200 --warmup 20 || exit 1
  arm p0b1_$r 1 --workload p0 --steps 200 --warmup 20 || exit 1
done
exit 0
