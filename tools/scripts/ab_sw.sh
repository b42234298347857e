#!/bin/bash
# SW probe (2M windows, 64 and 152 columns) for each library given (DRM_LIB), two rounds, same box.
set -o pipefail
for i in 1 2; do
  for lib in "$@"; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 200 python -u tools/scripts/sw_probe.py --windows 2000000 || exit 1
  done
done
