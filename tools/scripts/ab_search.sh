#!/bin/bash
# C5 search alone for each library given (DRM_LIB), two rounds, same box. Usage: bash tools/scripts/ab_search.sh TAG lib...
TAG=$1; shift
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/search_c5.py > gpurun_out/ab_$TAG.tmp 2>&1 || { tail -20 gpurun_out/ab_$TAG.tmp; exit 1; }
    grep -E "^search" gpurun_out/ab_$TAG.tmp
  done
done
