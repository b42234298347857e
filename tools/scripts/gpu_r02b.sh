#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench_r02b.json 2> gpurun_out/bench_r02b.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_r02b.err; exit 1; }
cat gpurun_out/bench_r02b.json
DRM_SEARCH_STAMPS=1 timeout -k 10 300 python -u tools/scripts/stamps.py c5 > gpurun_out/stamps_c5.txt 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_c5.txt; exit 1; }
cat gpurun_out/stamps_c5.txt
