#!/bin/bash
# Round 6: upper-level links as 16-B records carrying their node's list offset, and the entry point's top list held in
# registers per wave (current build) vs the build before it (ab_live/base.so): the search parity tests first, then the
# C5 search A/B, two rounds on one box.
set -o pipefail
mkdir -p gpurun_out/r06_ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tie_fixtures.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "search or broadcast or clone or tie" > gpurun_out/r06_ab/parity_upper.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error|assert" gpurun_out/r06_ab/parity_upper.log | head -20; tail -5 gpurun_out/r06_ab/parity_upper.log; exit 1; }
tail -1 gpurun_out/r06_ab/parity_upper.log
bash tools/scripts/ab_search.sh r06upper ab_live/base.so deepreadmapper_amd/libdrm_hip.so | tee gpurun_out/r06_ab/ab_search_upper.txt
