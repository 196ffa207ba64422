#!/bin/bash
# round 5: kernel trace of the S1 step on this tree (rocprofv3 --kernel-trace --stats); SERIAL=1: the branch
# stream and the side-stream weight gradients off (every kernel alone on the chip)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; OUT="$GRAFT_REPO_ROOT/gpurun_out"; export TMPDIR=/tmp
rm -rf "$OUT/s1prof"
cat > "$OUT/s1ser.py" <<'PY'
import os, runpy, sys
sys.argv = ["bench.py"] + sys.argv[1:]
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "endoscopy-image-classification_amd"))
if os.environ.get("SERIAL") == "1":
    os.environ["ENDOSSL_OVERLAP"] = "0"
    import endossl.conformer as c
    c.CONV_DW_SIDE = False
    c.BRANCH_STREAMS = False
runpy.run_path(os.path.join(os.environ["GRAFT_REPO_ROOT"], "bench.py"), run_name="__main__")
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/s1prof" -o run --output-format csv -- python3 "$OUT/s1ser.py" --workload s1 --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/s1prof.log" 2>&1; echo "s1prof rc=$?"
