#!/bin/bash
# bench.py --gpus 2 self-launch + --allreduce auto on a one-GPU box (both ranks on cuda:0 over gloo,
# 2 hardware queues per process): plumbing only
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export ENDOSSL_DIST_BACKEND=gloo ENDOSSL_SHARE_DEVICE=1 GPU_MAX_HW_QUEUES=2
timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/dp2auto.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/dp2auto.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("allreduce_form"), d.get("allreduce_choice"), d.get("allreduce_other_form",{}).get("ms_per_step"))'
exit $rc
