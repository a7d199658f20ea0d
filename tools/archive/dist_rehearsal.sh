#!/bin/bash
# Two ranks of bench.py on the one GPU of a box (torchrun, gloo for the
# collectives: RCCL refuses two ranks on one device), every sub-measurement
# at small step counts: rehearses the N>1 control flow of the driver's
# scaling run (barriers, max-over-ranks, logit all-gather + video score).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
FAC_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03_dist2.log 2>&1 || { tail -30 gpurun_out/r03_dist2.log; exit 1; }
tail -1 gpurun_out/r03_dist2.log | cut -c1-900
