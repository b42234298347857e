#!/bin/bash
# Profile of the GRU read encoder alone (tools/scripts/enc_bench.py, 1.25M tagged 150 bp reads): kernel-trace stats,
# then separate PMC passes (never combined with traces; per-block counter limits respected). Usage: profile_enc.sh TAG
set -u
TAG=${1:-enc}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
RUN="python3 tools/scripts/enc_bench.py 1250000"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $RUN > $OUT/trace.out 2> $OUT/trace.err || { echo "trace pass failed"; tail -5 $OUT/trace.err; exit 1; }
cat $OUT/trace.out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set -d $OUT/pmc$i -o run --output-format csv -- $RUN > $OUT/pmc${i}.out 2> $OUT/pmc${i}.err || { echo "pmc pass $i failed ($set)"; tail -3 $OUT/pmc${i}.err; exit 1; }
  echo "pass $i done"
done
python3 tools/scripts/summarize_profile.py $OUT > $OUT/summary.txt && grep -E "gru" $OUT/summary.txt | cut -c1-500
