#!/bin/bash
# GPU box: C5 search timing of several builds, alternating (no tests). Usage: gpu_ab_search_only.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for lib in "$@"; do echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done; done
