#!/bin/bash
# GPU box: the parity subset with an alternate library build (DRM_LIB; the CLI tests still load the in-tree build),
# then a C5 search A/B. Usage: gpu_ab_lib_tests.sh test.so lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
DRM_LIB=$PWD/$T timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_builder.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not cli and not flat" > gpurun_out/ab_lib_tests.log 2>&1 || { tail -30 gpurun_out/ab_lib_tests.log; exit 1; }
tail -1 gpurun_out/ab_lib_tests.log
for r in 1 2; do for lib in "$@"; do echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done; done
