#!/bin/bash
# S1 with every stream serialised (branch streams and the weight-gradient side stream off): per-kernel
# isolated times under rocprofv3, plus the serial and default step times
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-300; return $rc; }
ENDOSSL_BRANCH_STREAMS=0 ENDOSSL_CONV_DW_SIDE=0 run s1ser 300 python bench.py --workload s1 --steps 3 --warmup 2 || exit 1
ENDOSSL_BRANCH_STREAMS=0 ENDOSSL_CONV_DW_SIDE=0 run s1prof 400 rocprofv3 --kernel-trace --stats -d "$OUT/s1prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload s1 --steps 2 --warmup 1 || exit 1
exit 0
