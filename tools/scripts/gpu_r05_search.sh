#!/bin/bash
# Round-5 search iteration on one GPU box: the search parity tests (C1, syn20k, tie fixtures, log compaction), the
# C5 search A/B of the given libraries (same box, alternating), then the C5 512-read oracle check.
# Usage: bash tools/scripts/gpu_r05_search.sh TAG lib...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py -k "search or faiss" \
  > gpurun_out/${TAG}_parity.log 2>&1 || { tail -40 gpurun_out/${TAG}_parity.log; exit 1; }
tail -2 gpurun_out/${TAG}_parity.log
bash tools/scripts/ab_search.sh $TAG "$@" | tee gpurun_out/ab_${TAG}.txt || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_gpu_c5.py -k "search_and_rerank" \
  > gpurun_out/${TAG}_c5.log 2>&1 || { tail -40 gpurun_out/${TAG}_c5.log; exit 1; }
tail -2 gpurun_out/${TAG}_c5.log
