#!/bin/bash
# Round 4 GPU timing, part A: C5 search alone, new vs round-3 library (same box, alternating), then the stamps.
TAG=${TAG:-r04d}
set -o pipefail
mkdir -p gpurun_out
for lib in deepreadmapper_amd/libdrm_hip.so ab/libdrm_hip_r03.so deepreadmapper_amd/libdrm_hip.so ab/libdrm_hip_r03.so; do
  echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/search_c5.py > gpurun_out/search_c5_$TAG.tmp 2>&1 || { tail -20 gpurun_out/search_c5_$TAG.tmp; exit 1; }
  grep -E "^search" gpurun_out/search_c5_$TAG.tmp
done
DRM_SEARCH_STAMPS=1 timeout -k 10 300 python -u tools/scripts/stamps.py c5gru 2>&1 | grep -v "^\[bench\]\|^\[synth\]" > gpurun_out/stamps_c5gru_$TAG.txt; rc=$?; cat gpurun_out/stamps_c5gru_$TAG.txt; exit $rc
