#!/bin/bash
# GPU box: A/B of SW builds on the random-window probe (tools/scripts/sw_waves_probe.py), then the search
# kernel's section stamps at C5 (GRU). Usage: gpu_r03_ab_sw.sh lib1.so lib2.so
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in "$@"; do
    echo "== $lib"
    DRM_LIB=$PWD/$lib timeout -k 10 200 python -u tools/scripts/sw_waves_probe.py --waves 0 --windows 2000000 || exit 1
  done
done
DRM_SEARCH_STAMPS=1 timeout -k 10 600 python -u tools/scripts/stamps.py c5gru 2>&1 | grep -v "^\[bench\]\|^\[synth\]"
