#!/bin/bash
# GPU box: parity tests, then one bench line (optionally with section stamps). Usage: gpu_check.sh <tag> [--stamps] [--cpu]
set -e
TAG=${1:-x}; shift || true
STAMPS=0; CPU=--no-cpu
for a in "$@"; do case $a in --stamps) STAMPS=1;; --cpu) CPU=;; esac; done
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 600 python bench.py $CPU --steps 5 --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));b=d['breakdown'];print('value',d['value'],'search',b['search_ms'],'sw',b['sw_rerank_ms'],'frac',d['roofline']['frac'],'cpu',d['cpu_baseline'])"
if [ $STAMPS = 1 ]; then
  DRM_SEARCH_STAMPS=1 timeout -k 10 300 python tools/scripts/stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 || { echo STAMPS_FAILED; tail -20 gpurun_out/stamps_$TAG.txt; exit 1; }
  cat gpurun_out/stamps_$TAG.txt
fi
