#!/bin/bash
# Round 6, verdict items 1 + 3: the gated row load's parity on the small fixtures, then its price (chase probe at
# 1/2/3 lines, C5 valid-link histogram, hop-weighted line counts from the stamped kernel), a same-box A/B of the C5
# search against the round-5 library (ab_live/r05.so), and the FETCH_SIZE calibration on the chase kernel's known bytes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/r06_price
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "search" > $OUT/parity.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error|assert" $OUT/parity.log | head -20; tail -5 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
timeout -k 10 500 python -u tools/scripts/price_rows.py > $OUT/price_rows.txt 2> $OUT/price_rows.err || { echo PRICE_FAILED; tail -20 $OUT/price_rows.err; exit 1; }
cut -c1-400 $OUT/price_rows.txt
DRM_SEARCH_STAMPS=1 timeout -k 10 300 python -u tools/scripts/stamps.py c5gru > $OUT/stamps.txt 2> $OUT/stamps.err || { echo STAMPS_FAILED; tail -20 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.txt
bash tools/scripts/ab_search.sh r06gate ab_live/r05.so deepreadmapper_amd/libdrm_hip.so | tee $OUT/ab_search_gate.txt || { echo AB_FAILED; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- python3 tools/scripts/chase_calib.py run > $OUT/calib_run.txt 2> $OUT/calib.err || { echo CALIB_FAILED; tail -5 $OUT/calib.err; exit 1; }
python3 tools/scripts/chase_calib.py parse $OUT/calib | tee $OUT/calib.txt
