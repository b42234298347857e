#!/bin/bash
# One GPU box: the GPU suite, smoke(), the default bench (C5) and the C4 search-only bench (K = 128 and 5).
# Usage: TAG=r03x bash tools/scripts/gpu_r03b_full.sh
TAG=${TAG:-r03}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_${TAG}_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c5.json'));b=d['breakdown'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', d['roofline']['frac'], 'sw frac', d['sw_roofline']['frac'])"
timeout -k 10 900 python -u bench.py --workload c4 --no-cpu > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err || { echo BENCH_C4_FAILED; tail -20 gpurun_out/bench_${TAG}_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c4.json'));print('c4', d['value'], d['ms_per_step'], 'k5', d['k5'])"
