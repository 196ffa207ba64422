#!/bin/bash
# round-6 final confirm, in two calls (gpurun's 20-minute limit):
#   PART=1: the GPU suite, smoke(), the default F1 bench line (with the CPU baseline)
#   PART=2: S1 / C1 / P0 / N = 8 shard lines, a rocprofv3 --kernel-trace --stats run of the F1 bench, the step
#           counters (scripts/step_counters.py) and the FETCH/WRITE passes for roofline.traffic
#           (scripts/pmc_layer_bytes.py) -- the summaries are written into profiles/ from gpurun_out/ afterwards
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400; return $rc; }
if [ "${PART:-1}" = 1 ]; then
  run suite 800 python -u -m pytest -q -rf -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu tests/ || exit 1
  run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  run bench 300 python -u bench.py || exit 1
  exit 0
fi
run s1 300 python -u bench.py --workload s1 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
run c1 200 python -u bench.py --workload c1 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
run p0 200 python -u bench.py --workload p0 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
run shard 200 python -u bench.py --batch 8 --steps 50 --warmup 10 --no-cpu-baseline || exit 1
rm -rf "$OUT/prof"
run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline || exit 1
TAG=r06 bash scripts/gpu_step_counters.sh > "$OUT/cnt.log" 2>&1; echo "counters rc=$?"; tail -2 "$OUT/cnt.log"
bash scripts/gpu_pmc_step.sh > "$OUT/pstep.log" 2>&1; echo "pmc step rc=$?"; tail -2 "$OUT/pstep.log"
exit 0
