#!/bin/bash
# rocprofv3 kernel-trace summaries of the C1 (CoMatch) and S1 (SemiFormer) bench workloads.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for w in ${WL:-c1 s1}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$w" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 3 --warmup 1 > gpurun_out/prof_$w.log 2>&1 || exit $?
  tail -1 gpurun_out/prof_$w.log
done
