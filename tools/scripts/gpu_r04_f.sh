#!/bin/bash
# Round 4 GPU check after a search-kernel change: tie fixtures, the debug build on the tie + C1 fixtures, the parity
# file, then C5 search timing against the last committed build (ab/pq_prev.so) and the stamps. First failure ends it.
TAG=${TAG:-r04f}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 python -u tools/scripts/tie_search.py A B C D > gpurun_out/tie_$TAG.txt 2>&1; rc=$?; tail -5 gpurun_out/tie_$TAG.txt; [ $rc -eq 0 ] || exit 1
DRM_LIB=$PWD/ab/pqdbg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_search_committed_c1_fixture or test_search_tie_fixtures" > gpurun_out/gpu_dbg_$TAG.log 2>&1
rc=$?; grep -E "pq dbg|FAILED|Error" gpurun_out/gpu_dbg_$TAG.log | head -20; tail -1 gpurun_out/gpu_dbg_$TAG.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_$TAG.log | head -20; tail -5 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
for lib in deepreadmapper_amd/libdrm_hip.so ab/pq_prev.so deepreadmapper_amd/libdrm_hip.so ab/pq_prev.so; do
  echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/search_c5.py > gpurun_out/search_c5_$TAG.tmp 2>&1 || { tail -20 gpurun_out/search_c5_$TAG.tmp; exit 1; }
  grep -E "^search" gpurun_out/search_c5_$TAG.tmp
done
DRM_SEARCH_STAMPS=1 timeout -k 10 300 python -u tools/scripts/stamps.py c5gru 2>&1 | grep -v "^\[bench\]\|^\[synth\]" > gpurun_out/stamps_c5gru_$TAG.txt; rc=$?; cat gpurun_out/stamps_c5gru_$TAG.txt; exit $rc
