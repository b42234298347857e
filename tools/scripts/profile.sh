#!/bin/bash
# Profiles bench.py on the GPU box: kernel-trace stats + separate PMC passes (never combined with
# sys/runtime traces). Usage: bash tools/scripts/profile.sh <tag> [extra bench args]
set -u
TAG=${1:-r01}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python3 bench.py --no-cpu --no-host-path --steps 2 --warmup 1 $*"
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
# workload cache (index build etc.) outside the profiler
timeout -k 10 600 $BENCH > $OUT/warm.json 2> $OUT/warm.err || { echo "warm-up run failed"; tail -5 $OUT/warm.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $BENCH > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { echo "trace pass failed"; tail -5 $OUT/trace_bench.err; exit 1; }
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- $BENCH > $OUT/pmc${i}_bench.json 2> $OUT/pmc${i}.err || { echo "pmc pass $i failed ($set)"; tail -3 $OUT/pmc${i}.err; }
done
find $OUT -name "*.csv" | head -20
python3 tools/scripts/summarize_profile.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
