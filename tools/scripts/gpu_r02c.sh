#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r02c.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests_r02c.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r02c.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload c3 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err || { echo BENCH2_FAILED; tail -30 gpurun_out/bench_2rank.err; exit 1; }
cat gpurun_out/bench_2rank.json
