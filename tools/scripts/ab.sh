#!/bin/bash
# A/B kernel variants on one GPU box: alternates bench runs over the given in-tree .so builds.
# Usage: bash tools/scripts/ab.sh ROUNDS lib1.so lib2.so ...   (prints search / SW ms per run)
# (extra bench arguments in $BENCH_ARGS, e.g. BENCH_ARGS="--index flat")
set -e
R=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --steps 1 --warmup 1 ${BENCH_ARGS:-} > /dev/null 2>&1 # builds the workload cache
for r in $(seq $R); do
  for lib in "$@"; do
    DRM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/ab.json 2>/dev/null
    python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));b=d['breakdown'];print(sys.argv[1], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'])" $lib
  done
done
