#!/bin/bash
# Round 6 final call A: encoder occupancy A/B (layer 1 at 4 waves per SIMD vs the default 3), then smoke, the GPU suite,
# the profile and the default bench line of the final build (gpu_r06_final.sh with EXTRA=0).
set -o pipefail
mkdir -p gpurun_out/r06_final
for i in 1 2; do
  for lib in deepreadmapper_amd/libdrm_hip.so ab_live/encl1w4.so; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/enc_bench.py 1250000 2>&1 | tee -a gpurun_out/r06_final/ab_enc_l1waves.txt | grep encoder || exit 1
  done
done
EXTRA=0 bash tools/scripts/gpu_r06_final.sh
