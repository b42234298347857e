#!/bin/bash
# GRU read encoder: GPU tests + timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_enc_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_enc_tests.log; exit 1; }
grep -E "err|passed|failed" gpurun_out/gpu_enc_tests.log | tail -8
timeout -k 10 300 python -u tools/scripts/enc_bench.py ${ENC_N:-1250000} > gpurun_out/enc_bench.txt 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/enc_bench.txt; exit 1; }
cat gpurun_out/enc_bench.txt
