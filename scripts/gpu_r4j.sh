#!/bin/bash
# round-4 evidence: N = 8 shard A/B (attention-backward variants), wgrad SQ counters, S1 and F1 kernel traces
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
bash scripts/gpu_ab_shard.sh || exit 1
bash scripts/gpu_pmc_wgrad.sh || exit 1
bash scripts/gpu_s1prof.sh || exit 1
rm -rf "$OUT/f1prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/f1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/f1prof.log" 2>&1; rc=$?; echo "f1prof rc=$rc"; tail -1 "$OUT/f1prof.log" | cut -c1-300
exit $rc
