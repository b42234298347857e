#!/bin/bash
# GPU box: SW parity tests, then the co-residency probe at C5 (tools/scripts/coresident_c5.py). Usage: gpu_r03_co.sh TAG [probe args]
set -o pipefail
TAG=${1:-r03}; shift || true
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dynamic.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 900 python -u tools/scripts/coresident_c5.py "$@" > gpurun_out/${TAG}_co.log 2>&1
rc=$?; grep -v "^\[bench\]\|^\[synth\]" gpurun_out/${TAG}_co.log | tail -30; exit $rc
