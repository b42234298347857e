#!/bin/bash
# Round-6 profile of the default bench (C5, GRU): kernel-trace stats pass + separate PMC passes (never combined with
# traces; per-block counter limits of MI355X_MICROARCH.md respected). Usage: bash tools/scripts/profile_r06.sh TAG
set -u
TAG=${1:-r06}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python3 bench.py --no-cpu --no-host-path --no-encoder --no-l2 --steps 2 --warmup 1"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $BENCH > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo "trace pass failed"; tail -5 $OUT/trace_bench.err; exit 1; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- $BENCH > $OUT/pmc${i}_bench.json 2> $OUT/pmc${i}.err || { echo "pmc pass $i failed ($set)"; tail -3 $OUT/pmc${i}.err; exit 1; }
  echo "pass $i done"
done
python3 tools/scripts/summarize_profile.py $OUT > $OUT/summary.txt && grep -E "hnsw_pq_fast|sw_score_f16|steady" $OUT/summary.txt | cut -c1-400
