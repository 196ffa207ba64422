#!/bin/bash
# round 5: re-run the reworked loss checks, then a single-stream F1 kernel profile (ENDOSSL_OVERLAP=0: every
# kernel alone on the chip, its isolated time) for the per-kernel floor table
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-400; return $rc; }
PT="python -u -m pytest -v -rf -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
run sf 300 $PT tests/test_gpu_conformer.py -k semiformer_trainer -s; rc=$?; [ $rc -gt 1 ] && exit $rc
run par 400 $PT tests/test_gpu_parity.py -k full_size -s; rc=$?; [ $rc -gt 1 ] && exit $rc
rm -rf "$OUT/ser"
ENDOSSL_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/ser" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ser.log" 2>&1; rc=$?; echo "ser rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/prof_summary.py "$OUT/ser" r05_serial 7 > /dev/null && cp profiles/r05_serial_summary.md "$OUT/" ; exit 0
