#!/bin/bash
# Extra PMC passes (one rocprofv3 --pmc run per set, kernel-trace free). Usage: pmc_sets.sh TAG "SET1" "SET2" ...
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --no-cpu --steps 1 --warmup 1 > /dev/null 2>&1 # workload cache
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i failed ($set)"; tail -3 $OUT/p$i.err; }
done
python3 tools/scripts/summarize_profile.py $OUT > $OUT/summary.txt; grep -E "hnsw_pq_search_kernel|sw_score_f16" $OUT/summary.txt
