#!/bin/bash
# round 5: kernel trace of the C1 (CoMatch) step, every kernel alone on the chip (ENDOSSL_OVERLAP=0), and its
# bench line with the default two streams
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c1 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/c1.log" 2>&1 || exit 1
rm -rf "$OUT/c1prof"
ENDOSSL_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/c1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c1 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/c1prof.log" 2>&1; echo "c1prof rc=$?"
