#!/bin/bash
# round 5: grouped weight-gradient ring A/B (ENDOSSL_TN_GROUPED_RING 0 = 64x2, 1 = 32x4, 2 = 32x3; interleaved
# F1 bench runs on one box) and an N = 8 shard kernel trace for the per-stream timeline
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "big_grouped" > "$OUT/tk.log" 2>&1; rc=$?; tail -2 "$OUT/tk.log"; [ $rc -ne 0 ] && exit 1
for r in 1 2; do for ring in 0 1 2; do
  ENDOSSL_TN_GROUPED_RING=$ring timeout -k 10 200 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > "$OUT/ring${ring}_$r.log" 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/ring${ring}_$r.log') if l.startswith('{\"metric')][-1]); print('ring $ring round $r', d['ms_per_step'], d['roofline']['mean_launch_ms'], round(d['roofline']['frac'],4))"
done; done
rm -rf "$OUT/shard"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/shard" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch 8 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/shard.log" 2>&1; rc=$?; echo "shard rc=$rc"
[ $rc -ne 0 ] && exit $rc
f=$(ls "$OUT"/shard/*kernel_trace.csv "$OUT"/shard/*/*kernel_trace.csv 2>/dev/null | head -1); python3 scripts/step_timeline.py "$f" | tail -8
exit 0
