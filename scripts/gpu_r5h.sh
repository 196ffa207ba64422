#!/bin/bash
# round 5: the N = 8 shard (B = 8, mu = 7): two streams vs one (ENDOSSL_OVERLAP=0) vs hipGraph replay, interleaved;
# then the NT kernel families at the shard's shapes (gemm_bench --shard 8)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --batch 8 --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/sh_d$r.log" 2>&1 || exit 1
  ENDOSSL_OVERLAP=0 timeout -k 10 200 python -u bench.py --batch 8 --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/sh_s$r.log" 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --batch 8 --steps 200 --warmup 10 --no-cpu-baseline --graph on > "$OUT/sh_g$r.log" 2>&1 || exit 1
  echo "shard round $r: default $(ms $OUT/sh_d$r.log) serial $(ms $OUT/sh_s$r.log) graph $(ms $OUT/sh_g$r.log)"
done
timeout -k 10 400 python3 scripts/gemm_bench.py --shard 8 --variants=-1,0,2,5,10,11 --rounds 5 --iters 20 \
  --only qkv_fwd,proj_fwd,fc1_fwd,fc2_fwd,fc1_fwd_weak,fc2_dgrad,fc1_dgrad,proj_dgrad,qkv_dgrad,qkv_fwd_weak,proj_fwd_weak,fc2_fwd_weak \
  > "$OUT/shsweep.log" 2>&1; tail -12 "$OUT/shsweep.log"
