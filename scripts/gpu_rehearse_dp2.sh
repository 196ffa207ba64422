#!/bin/bash
# Rehearse bench.py's N = 2 path (torchrun, two ranks, per-block overlapped all-reduce) on a one-GPU
# box: both ranks on cuda:0 over gloo.  Checks the plumbing (rank-0 JSON line, barrier, max over
# ranks), not the scaling -- the driver's 8-GPU run over RCCL is the measurement.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
export ENDOSSL_DIST_BACKEND=gloo ENDOSSL_SHARE_DEVICE=1
for w in f1 c1; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --workload $w > gpurun_out/dp2_$w.log 2>&1; rc=$?
  echo "$w dp2 rc=$rc"; grep '"metric"' gpurun_out/dp2_$w.log | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
done
