#!/bin/bash
# Builds an alternate libdrm_hip.so with extra -D flags on the HIP kernels, for A/B timing on one box
# (tools/scripts/ab.sh, DRM_LIB). Usage: bash tools/scripts/build_variant.sh NAME [-DFLAG=V ...]
# -> ab_live/NAME.so (git-ignored, not gpurun-ignored: travels to the GPU box with the tree). Run `make` first.
set -e
NAME=$1; shift
ROCM=${ROCM:-/opt/rocm}
mkdir -p ab_live/$NAME.obj
FL="-O3 -std=c++17 -fPIC -Iinclude -Ideepreadmapper_amd/csrc -Wall -Wno-unused-result --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics $*"
for f in deepreadmapper_amd/csrc/*.hip; do
  k=$(basename $f .hip)
  $ROCM/bin/hipcc $FL -c $f -o ab_live/$NAME.obj/$k.o &
done
wait
$ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_live/$NAME.so ab_live/$NAME.obj/*.o build/capi.o build/exec.o build/faiss_io.o \
  build/formats.o build/builder.o build/embed.o build/hnswlib_io.o build/builder_flat.o build/encoder.o -L$ROCM/lib -lamdhip64 -lrccl -lgomp \
  -Wl,-soname,libdrm_hip.so
echo ab_live/$NAME.so
