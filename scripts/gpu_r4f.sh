#!/bin/bash
# round 4: BatchNorm / conv tests, then S1 A/B of the y-free BatchNorm backward (module constant) and of the
# conv weight-gradient split target, interleaved twice
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-600; return $rc; }
run tconf 400 python -u -m pytest tests/test_gpu_conformer.py -x -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
i=0
for r in 1 2; do for v in ${S1V:-endossl.conformer.BN_Y_FREE=0 endossl.conformer.BN_Y_FREE=1 es_set_conv_dw_target=256}; do
  i=$((i+1))
  timeout -k 10 300 python -u scripts/s1_knob_ab.py $(echo $v | tr "," " ") --workload s1 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/s1f_$i.log" 2>&1 || { tail -3 "$OUT/s1f_$i.log"; exit 1; }
  echo "$v: $(tail -1 $OUT/s1f_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
exit 0
