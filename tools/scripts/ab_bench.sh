#!/bin/bash
# C5 bench (device path only) for each library given (DRM_LIB), two rounds, same box: value, ms/step, search, SW.
# Usage: bash tools/scripts/ab_bench.sh TAG lib...
TAG=$1; shift
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    DRM_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu --no-host-path --no-encoder --no-l2 --steps 3 --warmup 1 > gpurun_out/ab_$TAG.json 2> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
    python -c "import json,sys;d=json.load(open('gpurun_out/ab_$TAG.json'));b=d['breakdown'];print(sys.argv[1], d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'])" $lib
  done
done
