#!/bin/bash
# Round 4 GPU check, part 1 (after the queue-fetch fix): the bounds-checked debug build on the tie and C1 fixtures,
# then the parity file with the default build; the first failure ends the call.
TAG=${TAG:-r04c}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 python -u tools/scripts/tie_search.py A B C D; rc=$?; echo "tie rc=$rc"; [ $rc -eq 0 ] || exit 1
DRM_LIB=$PWD/ab/pqdbg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_search_committed_c1_fixture or test_search_tie_fixtures" > gpurun_out/gpu_dbg_$TAG.log 2>&1
rc=$?; grep -E "pq dbg|PASSED|FAILED|Error" gpurun_out/gpu_dbg_$TAG.log | head -30; [ $rc -eq 0 ] || { echo DEBUG_FAILED; tail -30 gpurun_out/gpu_dbg_$TAG.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
grep -cE "PASSED" gpurun_out/gpu_tests_$TAG.log; tail -1 gpurun_out/gpu_tests_$TAG.log
