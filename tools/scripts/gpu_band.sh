#!/bin/bash
# Banded SW (opt-in): its GPU tests, then the SW probe at band 0 (full DP), 8, 16 and 32. First failure ends it.
TAG=${TAG:-band}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_band.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/band_tests_$TAG.log 2>&1 || { echo BAND_TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/band_tests_$TAG.log | head -20; tail -5 gpurun_out/band_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/band_tests_$TAG.log
for b in 0 8 16 32; do
  timeout -k 10 200 python -u tools/scripts/sw_probe.py --windows 2000000 --band $b >> gpurun_out/band_probe_$TAG.txt 2>&1 || { echo PROBE_FAILED; tail -5 gpurun_out/band_probe_$TAG.txt; exit 1; }
done
cat gpurun_out/band_probe_$TAG.txt
