#!/bin/bash
# A/B of library builds on the GRU encoder (enc_bench.py, 1.25M reads). Usage: ab_enc.sh ROUNDS lib1.so lib2.so ...
set -e
R=$1; shift
mkdir -p gpurun_out
for r in $(seq $R); do
  for lib in "$@"; do
    echo -n "$lib: "
    DRM_LIB=$PWD/$lib timeout -k 10 300 python tools/scripts/enc_bench.py 1250000 2>&1 | head -1
  done
done
