#!/bin/bash
# HBM read bytes (FETCH_SIZE, one counter pass each) of the C5 search alone for each library given (DRM_LIB).
# Usage: bash tools/scripts/gpu_fetch_ab.sh TAG lib...
TAG=$1; shift
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/fetch_$TAG
mkdir -p $OUT
i=0
for lib in "$@"; do
  i=$((i+1))
  DRM_LIB=$PWD/$lib timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/p$i -o run --output-format csv -- python3 tools/scripts/search_c5.py --reps 1 > $OUT/p$i.out 2> $OUT/p$i.err || { echo "pass $i failed ($lib)"; tail -3 $OUT/p$i.err; exit 1; }
  python3 - "$OUT/p$i/run_counter_collection.csv" "$lib" <<'PY'
import csv, collections, sys
v = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "hnsw_pq_fast_kernel<true, false, true, false>" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
        v[r["Dispatch_Id"]] += float(r["Counter_Value"])
print(sys.argv[2], "FETCH_SIZE GB per dispatch:", [round(x / 1e6, 2) for x in v.values()])
PY
  grep -E "^search" $OUT/p$i.out
done
