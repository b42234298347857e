#!/bin/bash
# executor change: executor/multi/CLI GPU tests, then the C3 CLI timing with the executor trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_dynamic.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_exec_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_exec_tests.log; exit 1; }
tail -1 gpurun_out/gpu_exec_tests.log
DRM_EXEC_VERBOSE=1 timeout -k 10 600 python -u tools/scripts/pipeline_c3.py > gpurun_out/pipeline_c3.txt 2>&1; rc=$?
grep -E "run |Search|device span|batch" gpurun_out/pipeline_c3.txt | tail -14
exit $rc
