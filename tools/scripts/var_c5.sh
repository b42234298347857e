#!/bin/bash
# C5 search time across processes on one box: per-step search / SW ms of N bench runs, with the GPU's
# clocks and temperature before each run
set -o pipefail
mkdir -p gpurun_out
N=${1:-4}
timeout -k 10 400 python bench.py --no-cpu --no-encoder --no-host-path --steps 1 --warmup 1 > /dev/null 2>gpurun_out/var_warm.err || { tail -5 gpurun_out/var_warm.err; exit 1; }
for r in $(seq $N); do
  rocm-smi --showtemp --showclocks 2>/dev/null | grep -E "sclk|mclk|Temperature \(Sensor junction" | tr -s ' ' | head -4
  DRM_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py --no-cpu --no-encoder --no-host-path --steps 6 --warmup 1 > gpurun_out/var.json 2> gpurun_out/var.err || { tail -5 gpurun_out/var.err; exit 1; }
  grep "per-step" gpurun_out/var.err
done
