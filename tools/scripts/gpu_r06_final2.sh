#!/bin/bash
# Round 6 closing call: smoke, the GPU suite and the default bench line of the final tree (no profile: the committed
# r06 profile is of the same kernels).
set -o pipefail
TAG=r06final2
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all_$TAG.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gpu_all_$TAG.log | head; tail -5 gpurun_out/gpu_all_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_all_$TAG.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));b=d['breakdown'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'host', d['host_path']['ms'], 'enc', d['encoder']['ms'], 'cpu', d['cpu_baseline']['value'], 'traffic', d['roofline']['traffic'])"
