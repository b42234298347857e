#!/bin/bash
# One GPU box's memory system vs the C5 search time (same build): clocks, memory latency microbenchmark, the C5
# search alone, and one PMC pass of translation / L2-latency counters over the search. Usage: box_diag.sh TAG
set -u
TAG=${1:-diag}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/diag_$TAG
mkdir -p $OUT
(rocm-smi --showclocks --showmemuse --showtemp --showpower 2>&1 | grep -v "^$" | head -40) > $OUT/smi.txt || true
timeout -k 10 300 ./tools/microbench/memlat > $OUT/memlat.txt 2>&1 || { echo memlat failed; cat $OUT/memlat.txt; exit 1; }
timeout -k 10 600 python3 -u tools/scripts/search_c5.py > $OUT/search.txt 2>&1 || { echo search failed; tail -5 $OUT/search.txt; exit 1; }
timeout -s KILL 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 tools/scripts/search_c5.py --reps 1 > $OUT/pmc_search.txt 2>&1 || echo "pmc pass failed"
python3 - $OUT <<'PY'
import collections, csv, glob, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/pmc/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "hnsw_pq_fast" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for disp, c in sorted(agg.items(), key=lambda x: int(x[0]))[-1:]:
    v = {k: sum(x) for k, x in c.items()}
    hit, miss = v.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0), v.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0)
    print(f"search dispatch {disp}: UTCL1 miss rate {miss / max(hit + miss, 1):.4f} ({miss:.3g} misses), "
          f"TCP->TCC read latency {v.get('TCP_TCC_READ_REQ_LATENCY_sum', 0) / max(v.get('TCP_TCC_READ_REQ_sum', 1), 1):.0f} cycles, "
          f"UTCL2 busy {v.get('GRBM_UTCL2_BUSY', 0) / max(v.get('GRBM_GUI_ACTIVE', 1), 1):.3f}")
PY
cat $OUT/smi.txt | grep -i -E "sclk|mclk|fclk|socclk|Temperature|Power" | head -12
cat $OUT/memlat.txt
grep "^search" $OUT/search.txt
