#!/bin/bash
# One GPU box: the GPU suite, smoke(), the default bench (C5), then a C5 search A/B of library builds.
# Usage: TAG=r03x bash tools/scripts/gpu_r03b_validate.sh [lib1.so lib2.so ...]
TAG=${TAG:-r03}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_${TAG}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c5.json'));b=d['breakdown'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', d['roofline']['frac'], 'sw frac', d['sw_roofline']['frac'])"
for lib in "$@"; do echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done
