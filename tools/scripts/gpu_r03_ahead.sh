#!/bin/bash
# GPU box: parity of a search-kernel variant library (DRM_LIB), then a same-box A/B at C5 against the baseline
# build, section stamps of the variant, and the visited-bitmap locality probe.
# Usage: bash tools/scripts/gpu_r03_ahead.sh ab/base.so ab/variant.so
BASE=$1; VAR=$2
set -o pipefail
mkdir -p gpurun_out
DRM_LIB=$PWD/$VAR timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py -x -q \
  --timeout 600 --timeout-method thread -m gpu -k "not flat and not coscheduled" > gpurun_out/ahead_tests.log 2>&1 || { tail -30 gpurun_out/ahead_tests.log; exit 1; }
tail -1 gpurun_out/ahead_tests.log
for r in 1 2; do for lib in $BASE $VAR; do echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done; done
for lib in $BASE $VAR; do echo "== $lib K=5"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py --k 5 2>&1 | grep "^search" || exit 1; done
DRM_LIB=$PWD/$VAR DRM_SEARCH_STAMPS=1 timeout -k 10 600 python -u tools/scripts/stamps.py c5gru > gpurun_out/ahead_stamps.txt 2>&1 || { tail -5 gpurun_out/ahead_stamps.txt; exit 1; }
cat gpurun_out/ahead_stamps.txt
timeout -k 10 600 python -u tools/scripts/vis_locality.py > gpurun_out/vis_locality.txt 2>&1 || { tail -5 gpurun_out/vis_locality.txt; exit 1; }
cat gpurun_out/vis_locality.txt
