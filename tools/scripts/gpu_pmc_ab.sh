#!/bin/bash
# Search A/B (ab_search.sh, two rounds) of the libraries given, then one SQ counter pass (instructions, waits) of the C5
# search for each (DRM_LIB). Usage: bash tools/scripts/gpu_pmc_ab.sh TAG lib...
TAG=$1; shift
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
bash tools/scripts/ab_search.sh $TAG "$@" > gpurun_out/ab_search_$TAG.txt 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/ab_search_$TAG.txt; exit 1; }
cat gpurun_out/ab_search_$TAG.txt
OUT=gpurun_out/pmcab_$TAG
mkdir -p $OUT
i=0
for lib in "$@"; do
  i=$((i+1))
  DRM_LIB=$PWD/$lib timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/p$i -o run --output-format csv -- python3 tools/scripts/search_c5.py --reps 1 > $OUT/p$i.out 2> $OUT/p$i.err || { echo "pmc pass $i failed ($lib)"; tail -3 $OUT/p$i.err; exit 1; }
  python3 - "$OUT/p$i/run_counter_collection.csv" "$lib" <<'PY'
import csv, collections, sys
v = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "hnsw_pq_fast_kernel<true, false, true, false>" in r["Kernel_Name"]:
        v[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
for d, c in v.items():
    print(sys.argv[2], "dispatch", d, " ".join(f"{k}={x:.4g}" for k, x in sorted(c.items())))
PY
done
