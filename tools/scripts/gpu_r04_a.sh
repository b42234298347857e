#!/bin/bash
# Round 4, first GPU check: the parity tests (heap-visited lean search, three-row SW DP), the C5 search alone
# (new library vs the round-3 library, same box, alternating), the SW probe (three rows vs two rows in flight),
# then a short C5 bench.
TAG=${TAG:-r04a}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
for i in 1 2; do
  for lib in deepreadmapper_amd/libdrm_hip.so ab/libdrm_hip_r03.so; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep -E "^search|Error|error" || exit 1
  done
done
for i in 1 2; do
  for lib in deepreadmapper_amd/libdrm_hip.so ab/sw_r2.so ab/sw_r4pf1.so ab/sw_r5pf1.so; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/sw_waves_probe.py --waves 0 --windows 2000000 || exit 1
  done
done
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 --no-host-path --no-encoder --no-l2 --cpu-budget 5 > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_${TAG}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c5.json'));b=d['breakdown'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', d['roofline']['frac'], 'ndis', b['ndis_mean'], 'computed', b.get('distances_computed_mean'), 'nhops', b['nhops_mean'])"
