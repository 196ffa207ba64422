#!/bin/bash
# S1 A/B of the conv weight-gradient split target (es_set_conv_dw_target), interleaved twice, then the S1 profile
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
i=0
for r in 1 2; do for v in ${DWV:-2048 1024 512}; do
  i=$((i+1))
  timeout -k 10 300 python -u scripts/s1_knob_ab.py es_set_conv_dw_target=$v --workload s1 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/s1ab_$i.log" 2>&1 || { tail -3 "$OUT/s1ab_$i.log"; exit 1; }
  echo "dw_target $v: $(tail -1 $OUT/s1ab_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done; done
if [ -n "$PROF" ]; then bash scripts/gpu_s1prof.sh || exit 1; fi
exit 0
