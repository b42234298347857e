#!/bin/bash
# Round 6 batch 2: checksum hazard probe (item 2), salted chase pricing + FETCH_SIZE calibration (items 1, 3),
# encoder profile (item 5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/r06_b2
mkdir -p $OUT
timeout -k 10 300 python -u tools/scripts/checksum_hazard.py > $OUT/checksum_hazard.txt 2>&1 || { echo HAZARD_FAILED; tail -20 $OUT/checksum_hazard.txt; exit 1; }
cat $OUT/checksum_hazard.txt
timeout -k 10 300 python -u tools/scripts/price_rows.py --no-hist > $OUT/chase_salted.txt 2>&1 || { echo PRICE_FAILED; tail -20 $OUT/chase_salted.txt; exit 1; }
cat $OUT/chase_salted.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- python3 tools/scripts/chase_calib.py run > $OUT/calib_run.txt 2> $OUT/calib.err || { echo CALIB_FAILED; tail -5 $OUT/calib.err; exit 1; }
python3 tools/scripts/chase_calib.py parse $OUT/calib | tee $OUT/calib.txt
bash tools/scripts/profile_enc.sh r06enc || { echo ENC_PROFILE_FAILED; exit 1; }
# item 6: the drop-in host path, new schedule (kernels one after the other, ramped first/last batches) vs the
# round-2 overlap schedule, same box
for ov in 0 1 0; do
  DRM_EXEC_OVERLAP=$ov timeout -k 10 600 python -u bench.py --no-cpu --no-encoder --no-l2 --steps 3 --warmup 1 > $OUT/bench_hostpath_ov$ov.json 2> $OUT/bench_hostpath_ov$ov.err || { echo BENCH_FAILED; tail -20 $OUT/bench_hostpath_ov$ov.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_hostpath_ov$ov.json'));h=d['host_path'];print('overlap=$ov', 'device step', d['ms_per_step'], 'host path ms', h['ms'], 'span', h['device_span_ms'], 'ratio', round(h['ms']/d['ms_per_step'],4), h['status_ok'])"
done
