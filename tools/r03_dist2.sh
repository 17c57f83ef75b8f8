#!/bin/bash
# Rehearsal of `bench.py --gpus 2` on a one-GPU box: torchrun with 2 ranks, both on device 0
# (SKV_BENCH_SHARE_DEVICE=1), gloo barrier + max-over-ranks reduction, each rank its own compaction.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03; mkdir -p $O
SKV_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-host-path \
  > $O/dist2.log 2>&1 || { tail -30 $O/dist2.log; exit 1; }
grep '^{' $O/dist2.log | tail -1 | cut -c1-700
