#!/bin/bash
# Round 4: the co-scheduled step (search(b) beside SW(b-1), capped grids) against the sequential step, same box.
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-cpu --no-host-path --no-encoder --no-l2 --steps 3 --warmup 1"
timeout -k 10 400 $B > gpurun_out/co_seq.json 2> gpurun_out/co_seq.err || { tail -5 gpurun_out/co_seq.err; exit 1; }
for cfg in "4 12 4" "4 8 4" "8 12 4"; do
  set -- $cfg
  DRM_CO_BATCHES=$1 DRM_CO_SEARCH_WAVES=$2 DRM_CO_SW_WAVES=$3 timeout -k 10 400 $B --co > gpurun_out/co_$1_$2_$3.json 2> gpurun_out/co_$1_$2_$3.err || { tail -5 gpurun_out/co_$1_$2_$3.err; exit 1; }
done
for f in gpurun_out/co_seq.json gpurun_out/co_4_12_4.json gpurun_out/co_4_8_4.json gpurun_out/co_8_12_4.json; do
  python -c "import json,sys;d=json.load(open('$f'));b=d['breakdown'];print('$f', round(d['value']), d['ms_per_step'], b.get('search_ms'), b.get('sw_rerank_ms'), b.get('schedule'))"
done
