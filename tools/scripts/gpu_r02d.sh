#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_r02d_c5.json 2> gpurun_out/bench_r02d_c5.err || { echo C5_FAILED; tail -20 gpurun_out/bench_r02d_c5.err; exit 1; }
DRM_SEARCH_STAMPS=1 timeout -k 10 300 python -u tools/scripts/stamps.py c5 > gpurun_out/stamps_c5b.txt 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_c5b.txt; exit 1; }
cat gpurun_out/stamps_c5b.txt
timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/bench_r02d_c4.json 2> gpurun_out/bench_r02d_c4.err || { echo C4_FAILED; tail -20 gpurun_out/bench_r02d_c4.err; exit 1; }
cat gpurun_out/bench_r02d_c4.json
