#!/bin/bash
# Round 4 GPU check, staged so that a failure ends the call: (1) the bounds-checked debug build of the lean search
# on the tie fixtures and the C1 fixture; (2) the parity file with the default build; (3) C5 search alone, new vs
# round-3 library (alternating); (4) SW probe, rows in flight 3 (default) / 2 / 4 / 5; (5) stamps of the C5 search;
# (6) a short C5 bench.
TAG=${TAG:-r04b}
set -o pipefail
mkdir -p gpurun_out
DRM_LIB=$PWD/ab/pqdbg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "test_search_committed_c1_fixture or test_search_tie_fixtures" > gpurun_out/gpu_dbg_$TAG.log 2>&1
rc=$?; grep -E "pq dbg|PASSED|FAILED|Error" gpurun_out/gpu_dbg_$TAG.log | head -30; [ $rc -eq 0 ] || { echo DEBUG_FAILED; tail -30 gpurun_out/gpu_dbg_$TAG.log; exit 1; }
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
DRM_SEARCH_STAMPS=1 timeout -k 10 600 python -u tools/scripts/stamps.py c5gru 2>&1 | grep -v "^\[bench\]\|^\[synth\]" | tee gpurun_out/stamps_c5gru_$TAG.txt
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 --no-host-path --no-encoder --no-l2 --cpu-budget 5 > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_${TAG}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c5.json'));b=d['breakdown'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', d['roofline']['frac'], 'ndis', b['ndis_mean'], 'computed', b.get('distances_computed_mean'), 'nhops', b['nhops_mean'])"
