#!/bin/bash
# PMC of the C5 search alone (tools/scripts/search_c5.py), one counter pass (SQ block, <= 8 counters), plus an A/B of
# DRM_LIB variants given as arguments. Usage: bash tools/scripts/gpu_pmc_search.sh TAG [variant.so ...]
TAG=${1:-pmcs}; shift
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_search_$TAG
mkdir -p $OUT
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc1 -o run --output-format csv -- python3 tools/scripts/search_c5.py > $OUT/pmc1.out 2> $OUT/pmc1.err || { echo "pmc pass failed"; tail -3 $OUT/pmc1.err; exit 1; }
python3 tools/scripts/summarize_profile.py $OUT > $OUT/summary.txt && grep -E "hnsw_pq_fast" $OUT/summary.txt | cut -c1-600
for lib in deepreadmapper_amd/libdrm_hip.so "$@" deepreadmapper_amd/libdrm_hip.so "$@"; do
  echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 300 python -u tools/scripts/search_c5.py > $OUT/ab.tmp 2>&1 || { tail -20 $OUT/ab.tmp; exit 1; }
  grep -E "^search" $OUT/ab.tmp
done
