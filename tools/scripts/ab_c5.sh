#!/bin/bash
# A/B of in-tree library builds on the C5 bench (and C3): search / SW ms per run. Usage: ab_c5.sh ROUNDS lib1.so lib2.so ...
set -e
R=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --steps 1 --warmup 1 > /dev/null 2>gpurun_out/ab_warm.err # C5 cache
timeout -k 10 300 python bench.py --no-cpu --steps 1 --warmup 1 --workload c3 > /dev/null 2>&1 # C3 cache
for r in $(seq $R); do
  for lib in "$@"; do
    for wl in c5 c3; do
      DRM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 --workload $wl > gpurun_out/ab.json 2>/dev/null
      python -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));b=d['breakdown'];print(sys.argv[1], sys.argv[2], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'ndis', b['ndis_mean'])" $lib $wl
    done
  done
done
