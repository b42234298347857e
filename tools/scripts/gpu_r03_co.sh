set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r03a_parity.log 2>&1 && \
timeout -k 10 900 python -u tools/scripts/coresident_c5.py > gpurun_out/r03a_co.log 2>&1
rc=$?; tail -5 gpurun_out/r03a_parity.log; cat gpurun_out/r03a_co.log | grep -v "^\[bench\]" | tail -30; exit $rc
