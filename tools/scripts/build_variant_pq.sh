#!/bin/bash
# Builds an alternate libdrm_hip.so whose search kernel file (hnsw_pq_fast.hip) gets extra compiler flags, linked with
# the current build/ objects of every other file, for A/B timing on one box (DRM_LIB). Run `make` first.
# Usage: bash tools/scripts/build_variant_pq.sh NAME [flag ...]  -> ab_live/NAME.so
# PQ_SRC=path builds that copy of the file instead (e.g. the previous commit's, from `git show`).
set -e
NAME=$1; shift
ROCM=${ROCM:-/opt/rocm}
mkdir -p ab_live
FL="-O3 -std=c++17 -fPIC -Iinclude -Ideepreadmapper_amd/csrc -Wall -Wno-unused-result --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics $*"
$ROCM/bin/hipcc $FL -c ${PQ_SRC:-deepreadmapper_amd/csrc/hnsw_pq_fast.hip} -o ab_live/$NAME.pq.o
OBJS=$(ls build/*.o | grep -v hnsw_pq_fast.o)
$ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_live/$NAME.so ab_live/$NAME.pq.o $OBJS -L$ROCM/lib -lamdhip64 -lrccl -lgomp \
  -Wl,-soname,libdrm_hip.so
rm -f ab_live/$NAME.pq.o
echo ab_live/$NAME.so
