#!/bin/bash
# grouped weight-gradient tests (timed form), then the bench under a kernel trace: the line's kernel-stamped
# roofline span and the trace's span of the same launches come from one process
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "big_grouped or cls_head" > "$OUT/tk.log" 2>&1; rc=$?; tail -2 "$OUT/tk.log"; [ $rc -ne 0 ] && exit 1
rm -rf "$OUT/f1prof2"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/f1prof2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/f1prof2.log" 2>&1; rc=$?; echo "prof rc=$rc"
grep '^{"metric"' "$OUT/f1prof2.log" | tail -1 > "$OUT/f1prof2_line.json"
python3 -c "import json; d=json.load(open('$OUT/f1prof2_line.json')); print(d['ms_per_step'], d['roofline']['mean_launch_ms'])"
exit $rc
