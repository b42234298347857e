#!/bin/bash
# Round 6 batch 3: the whole GPU suite on the current build (checksum fix, executor schedule, encoder strides), then
# a same-box A/B of the encoder against the build before the LDS stride change (ab_live/enc_base.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/r06_b3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_all.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" $OUT/gpu_all.log | head; tail -5 $OUT/gpu_all.log; exit 1; }
tail -1 $OUT/gpu_all.log
for i in 1 2; do
  for lib in ab_live/enc_base.so deepreadmapper_amd/libdrm_hip.so; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/enc_bench.py 1250000 2>&1 | tee -a $OUT/ab_enc.txt | grep encoder || exit 1
  done
done
