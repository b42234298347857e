#!/bin/bash
# GPU box: parity of a search-kernel variant library (DRM_LIB), then a same-box A/B at C5 against the baseline
# build, and section stamps of both (FIX128 stamped build).
# Usage: bash tools/scripts/gpu_r03_ahead.sh ab/base.so ab/variant.so
BASE=$1; VAR=$2
set -o pipefail
mkdir -p gpurun_out
DRM_LIB=$PWD/$VAR timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_c5.py -x -q \
  --timeout 600 --timeout-method thread -m gpu -k "not flat and not coscheduled" > gpurun_out/ahead_tests.log 2>&1 || { tail -30 gpurun_out/ahead_tests.log; exit 1; }
tail -1 gpurun_out/ahead_tests.log
for r in 1 2; do for lib in $BASE $VAR; do echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done; done
for lib in $BASE $VAR; do echo "== $lib K=5"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py --k 5 2>&1 | grep "^search" || exit 1; done
for lib in $BASE $VAR; do echo "== stamps $lib"; DRM_LIB=$PWD/$lib DRM_SEARCH_STAMPS=1 timeout -k 10 600 python -u tools/scripts/stamps.py c5gru 2>&1 | grep -v "^\[bench\]" || exit 1; done
