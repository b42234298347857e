#!/bin/bash
# A/B environment settings on one GPU box: bash tools/scripts/ab_env.sh ROUNDS "ENV1" "ENV2" ...
# (extra bench arguments in $BENCH_ARGS, e.g. BENCH_ARGS="--index flat")
set -e
R=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --steps 1 --warmup 1 ${BENCH_ARGS:-} > /dev/null 2>&1
for r in $(seq $R); do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/ab.json 2>/dev/null
    python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));b=d['breakdown'];print(sys.argv[1], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'fallbacks', b.get('tie_fallback_queries'))" "$e"
  done
done
