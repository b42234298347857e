#!/bin/bash
# N = 2 rehearsal of the metric's configuration (C5 per-GPU slice) on a one-GPU box: two ranks share the device
# (each with its own index replica, 2 x ~70 GB of the 288 GB), the gloo control plane, max-over-ranks timing; the
# RCCL gather needs one GPU per rank, so it is reported as skipped. Default legs, as the driver runs it (the L2 leg
# skips itself at N > 1, the CPU baseline runs at N = 1 only).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_2rank_${TAG:-r06}.json 2> gpurun_out/bench_2rank_${TAG:-r06}.err || { echo FAILED; tail -30 gpurun_out/bench_2rank_${TAG:-r06}.err; exit 1; }
cat gpurun_out/bench_2rank_${TAG:-r06}.json
