#!/bin/bash
# A/B of physically contiguous allocations (DRM_CONTIG mask: 1 index arrays, 2 visited bitmaps,
# 4 window table) on C5: search / SW ms per process, modes alternating. Usage: ab_contig.sh ROUNDS MODE...
set -o pipefail
mkdir -p gpurun_out
R=${1:-2}; shift
timeout -k 10 400 python bench.py --no-cpu --no-encoder --no-host-path --steps 1 --warmup 1 > /dev/null 2>gpurun_out/abc_warm.err || { tail -5 gpurun_out/abc_warm.err; exit 1; }
for r in $(seq $R); do
  for c in "$@"; do
    DRM_CONTIG=$c timeout -k 10 300 python bench.py --no-cpu --no-encoder --no-host-path --steps 4 --warmup 1 > gpurun_out/abc.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/abc.json'));b=d['breakdown'];print('contig', sys.argv[1], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'])" $c
  done
done
