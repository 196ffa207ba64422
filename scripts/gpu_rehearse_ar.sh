#!/bin/bash
# bench.py's N = 2 path on a one-GPU box (both ranks on cuda:0, gloo): single vs per-block overlapped
# gradient all-reduce, and the overlapped one with the engine's second stream off.  Plumbing only.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export ENDOSSL_DIST_BACKEND=gloo ENDOSSL_SHARE_DEVICE=1
for v in "ENDOSSL_OVERLAP_AR=1 ENDOSSL_OVERLAP=0" "ENDOSSL_OVERLAP_AR=1 ENDOSSL_OVERLAP=bwd" "ENDOSSL_OVERLAP_AR=1 ENDOSSL_OVERLAP=fwd"; do
  env $v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 2 --steps 4 --warmup 2 > gpurun_out/dp2_v.log 2>&1 || exit $?
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dp2_v.log)"
done
