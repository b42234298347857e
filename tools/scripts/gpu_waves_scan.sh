#!/bin/bash
# C5 search alone at 12 / 16 / 20 resident waves per CU (DRM_SEARCH_WAVES_PER_CU), same box.
set -o pipefail
mkdir -p gpurun_out
for w in 20 16 12 20; do
  echo "== waves/CU $w"; DRM_SEARCH_WAVES_PER_CU=$w timeout -k 10 300 python -u tools/scripts/search_c5.py > gpurun_out/waves_scan.tmp 2>&1 || { tail -20 gpurun_out/waves_scan.tmp; exit 1; }
  grep -E "^search" gpurun_out/waves_scan.tmp
done
