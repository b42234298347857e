#!/bin/bash
# GPU box: a pytest selection (-k expr) then the default bench without CPU baseline. Usage: gpu_quick.sh TAG "KEXPR" [bench args]
set -o pipefail
TAG=$1; K=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 900 python -u bench.py --no-cpu "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));b=d['breakdown'];print('value',d['value'],'search',b['search_ms'],'sw',b['sw_rerank_ms'],'frac',d['roofline']['frac'])"
