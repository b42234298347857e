#!/bin/bash
# GPU box: C5 per-GPU slice bench (GPU-built 50M-window index), verbose build timings.
# Usage: gpu_c5.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-c5}; shift || true
mkdir -p gpurun_out
DRM_BUILD_VERBOSE=1 timeout -k 10 1000 python -u bench.py --workload c5 "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
tail -12 gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
