#!/bin/bash
# Round 5 check: smoke, the whole GPU suite, the default bench line, then optional A/B runs (SW probe of the given
# libraries). First failure ends it. Usage: TAG=... bash tools/scripts/gpu_r05_full.sh [sw_lib ...]
TAG=${TAG:-r05}
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all_$TAG.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gpu_all_$TAG.log | head; tail -5 gpurun_out/gpu_all_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_all_$TAG.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));b=d['breakdown'];r=d['roofline'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', r['frac'], 'floor', r['latency_floor_ms'], r['frac_of_latency_floor'], 'cpu', d['cpu_baseline']['value'])"
if [ $# -gt 0 ]; then
  bash tools/scripts/ab_sw.sh "$@" > gpurun_out/ab_sw_$TAG.txt 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/ab_sw_$TAG.txt; exit 1; }
  cat gpurun_out/ab_sw_$TAG.txt
fi
