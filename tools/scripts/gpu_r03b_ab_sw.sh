#!/bin/bash
# GPU box: SW parity (KAT, C1 matrix, dense/sparse/dynamic reranks vs the oracle) with the default build, then an
# A/B of SW builds on the random-window probe (tools/scripts/sw_waves_probe.py). Usage: gpu_r03b_ab_sw.sh lib1.so lib2.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dynamic.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/ab_sw_tests.log 2>&1 || { tail -30 gpurun_out/ab_sw_tests.log; exit 1; }
tail -1 gpurun_out/ab_sw_tests.log
for r in 1 2; do
  for lib in "$@"; do
    echo "== $lib"
    DRM_LIB=$PWD/$lib timeout -k 10 200 python -u tools/scripts/sw_waves_probe.py --waves 0 --windows 2000000 || exit 1
  done
done
