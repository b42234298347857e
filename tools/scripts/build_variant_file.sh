#!/bin/bash
# Builds an alternate libdrm_hip.so in which one kernel file (FILE=csrc basename, e.g. sw_rerank) gets extra compiler
# flags, linked with the current build/ objects of every other file, for A/B timing on one box (DRM_LIB). Run `make`
# first. Usage: FILE=sw_rerank bash tools/scripts/build_variant_file.sh NAME [flag ...] -> ab_live/NAME.so
set -e
NAME=$1; shift
ROCM=${ROCM:-/opt/rocm}
: "${FILE:?FILE=<csrc basename> required}"
mkdir -p ab_live
FL="-O3 -std=c++17 -fPIC -Iinclude -Ideepreadmapper_amd/csrc -Wall -Wno-unused-result --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics $*"
$ROCM/bin/hipcc $FL -c ${SRC:-deepreadmapper_amd/csrc/$FILE.hip} -o ab_live/$NAME.$FILE.o
OBJS=$(ls build/*.o | grep -v "/$FILE.o")
$ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_live/$NAME.so ab_live/$NAME.$FILE.o $OBJS -L$ROCM/lib -lamdhip64 -lrccl -lgomp \
  -Wl,-soname,libdrm_hip.so
rm -f ab_live/$NAME.$FILE.o
echo ab_live/$NAME.so
