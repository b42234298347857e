#!/bin/bash
# search-kernel change: GPU parity suites, then a one-box A/B (C5 GRU, C3) against the previous build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_search_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_search_tests.log; exit 1; }
tail -2 gpurun_out/gpu_search_tests.log
timeout -k 10 1200 bash tools/scripts/ab_c5.sh ${AB_ROUNDS:-2} "$@" > gpurun_out/ab_search.txt 2>&1; rc=$?
cat gpurun_out/ab_search.txt
exit $rc
