#!/bin/bash
# GPU box: parity subset, then an A/B of search builds at C5 (tools/scripts/search_c5.py). Usage: gpu_r03_ab_search.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not c4 and not flat" > gpurun_out/ab_search_tests.log 2>&1 || { tail -30 gpurun_out/ab_search_tests.log; exit 1; }
tail -1 gpurun_out/ab_search_tests.log
for r in 1 2; do for lib in "$@"; do echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done; done
