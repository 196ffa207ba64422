#!/bin/bash
# F1 same-box A/B of two library builds: build/oldlib (A) vs the tree's (B), interleaved R times
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
for r in $(seq ${R:-3}); do
  ENDOSSL_LIB=$PWD/build/oldlib/libendossl_hip.so timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BARGS} > "$OUT/abl_a$r.log" 2>&1 || exit 1
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BARGS} > "$OUT/abl_b$r.log" 2>&1 || exit 1
  echo "old $(tail -1 $OUT/abl_a$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')  new $(tail -1 $OUT/abl_b$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
