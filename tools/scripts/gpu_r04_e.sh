#!/bin/bash
# Round 4 GPU timing, part B: SW probe with 3 (default) / 2 / 4 / 5 rows in flight (same box, twice), then the default
# bench (C5, N=1).
TAG=${TAG:-r04e}
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in deepreadmapper_amd/libdrm_hip.so ab/sw_r2.so ab/sw_r4pf1.so ab/sw_r5pf1.so; do
    echo "== $lib"; DRM_LIB=$PWD/$lib timeout -k 10 200 python -u tools/scripts/sw_waves_probe.py --waves 0 --windows 2000000 || exit 1
  done
done 2>&1 | tee gpurun_out/sw_probe_$TAG.txt
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
