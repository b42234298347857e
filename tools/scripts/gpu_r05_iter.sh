#!/bin/bash
# Round-5 search iteration: search parity tests on the in-tree build, C5 search A/B of the given libraries (same
# box, alternating), one SQ PMC pass and the section stamps of the in-tree build. Usage: gpu_r05_iter.sh TAG lib...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py -k "search or faiss" \
  > gpurun_out/${TAG}_parity.log 2>&1 || { tail -40 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
bash tools/scripts/ab_search.sh $TAG "$@" | tee gpurun_out/ab_${TAG}.txt || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_search_$TAG
mkdir -p $OUT
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/pmc1 -o run --output-format csv -- python3 tools/scripts/search_c5.py > $OUT/pmc1.out 2> $OUT/pmc1.err || { echo "pmc pass failed"; tail -3 $OUT/pmc1.err; exit 1; }
python3 tools/scripts/summarize_profile.py $OUT > $OUT/summary.txt && grep -E "hnsw_pq_fast" $OUT/summary.txt | cut -c1-400
DRM_SEARCH_STAMPS=1 timeout -k 10 300 python3 tools/scripts/stamps.py c5gru > gpurun_out/stamps_${TAG}.txt 2>&1 || { tail -5 gpurun_out/stamps_${TAG}.txt; exit 1; }
cat gpurun_out/stamps_${TAG}.txt | tail -16
