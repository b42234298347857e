#!/bin/bash
# Round 6: the encoder's tiles per launch against the chip's concurrent workgroups (3 per CU x 256 CUs = 768 = 384
# tiles x 2 directions): 2048 tiles per launch leave a third-full last round in every launch; 1920 / 2304 / 3072 are
# whole rounds. Two rounds, one box.
set -o pipefail
mkdir -p gpurun_out/r06_enc
for i in 1 2; do
  for t in 2048 1920 2304 3072; do
    echo "== DRM_ENC_TILES=$t"; DRM_ENC_TILES=$t timeout -k 10 300 python -u tools/scripts/enc_bench.py 1250000 2>&1 | tee -a gpurun_out/r06_enc/ab_enc_tiles.txt | grep encoder || exit 1
  done
done
