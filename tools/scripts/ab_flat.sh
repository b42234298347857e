#!/bin/bash
# flat (hnswlib fp32) kernel change: GPU flat parity tests, then A/B on C3-flat. Usage: ab_flat.sh ROUNDS lib1.so lib2.so ...
set -o pipefail
R=$1; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_scale.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_flat_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_flat_tests.log; exit 1; }
tail -1 gpurun_out/gpu_flat_tests.log
timeout -k 10 300 python bench.py --no-cpu --no-host-path --no-encoder --steps 1 --warmup 1 --workload c3 --index flat > /dev/null 2>&1
for r in $(seq $R); do
  for lib in "$@"; do
    DRM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-host-path --no-encoder --steps 5 --warmup 1 --workload c3 --index flat > gpurun_out/abf.json 2>/dev/null
    python -c "import json,sys;d=json.load(open('gpurun_out/abf.json'));b=d['breakdown'];print(sys.argv[1], 'search', b['search_ms'], 'frac', d['roofline']['frac'], 'ndis', b['ndis_mean'])" $lib
  done
done
