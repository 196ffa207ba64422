#!/bin/bash
# bench.py's N = 2 path on a one-GPU box (both ranks on cuda:0, gloo): the single post-backward all-reduce
# vs the per-block overlapped one, at the default hardware-queue count and at GPU_MAX_HW_QUEUES=2
# (hypothesis under test: two processes x (main + side + comm + gloo copy streams) oversubscribe the
# GPU's hardware queues, and the scheduler then time-slices whole queues).  Plumbing only.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export ENDOSSL_DIST_BACKEND=gloo ENDOSSL_SHARE_DEVICE=1
i=0
# measured (r02): single 103.5 ms/step, overlapped 3,488 ms, overlapped at GPU_MAX_HW_QUEUES=2 79.1 ms
# (the single all-reduce at 2 queues segfaulted both ranks at start-up once; not re-run)
for v in "ENDOSSL_OVERLAP_AR=0" "ENDOSSL_OVERLAP_AR=1" "ENDOSSL_OVERLAP_AR=1 GPU_MAX_HW_QUEUES=2"; do
  i=$((i+1))
  env $v timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29518 + i)) bench.py --gpus 2 --steps 4 --warmup 2 --scaling weak --no-cpu-baseline > gpurun_out/dp2_v$i.log 2>&1 || exit $?
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp2_v$i.log)"
done
