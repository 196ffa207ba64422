#!/bin/bash
# round 5: FixMatch hipGraph replay (--graph on) vs eager at F1 and the N = 8 shard on this tree (same box,
# interleaved), then a kernel trace of the graph-replayed P0 step
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
ms() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'])"; }
for r in 1 2; do
  for w in f1 sh; do
    case $w in f1) a="--steps 100 --warmup 5";; sh) a="--batch 8 --steps 50 --warmup 10";; esac
    line="$w r$r"
    for gr in off on; do
      timeout -k 10 200 python -u bench.py --no-cpu-baseline $a --graph $gr > "$OUT/z_$w$gr$r.log" 2>&1 || exit 1
      line="$line $gr $(ms $OUT/z_$w$gr$r.log)"
    done
    echo "$line"
  done
done
rm -rf "$OUT/p0prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p0prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload p0 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/p0prof.log" 2>&1; echo "p0prof rc=$?"
