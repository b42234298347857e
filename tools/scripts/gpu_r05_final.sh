#!/bin/bash
# Round 5 final measurement: smoke and the whole GPU suite (SUITE=0 skips them), the profile (kernel-trace stats +
# separate PMC passes) of the default bench, then the default bench line with the opt-in banded SW leg beside it.
# First failure ends it.
TAG=${TAG:-r05final}
set -o pipefail
mkdir -p gpurun_out
if [ "${SUITE:-1}" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all_$TAG.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gpu_all_$TAG.log | head; tail -5 gpurun_out/gpu_all_$TAG.log; exit 1; }
  tail -1 gpurun_out/gpu_all_$TAG.log
fi
bash tools/scripts/profile_r05.sh $TAG || { echo PROFILE_FAILED; exit 1; }
timeout -k 10 600 python -u bench.py --sw-band 16 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));b=d['breakdown'];r=d['roofline'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', r['frac'], 'floor', r['latency_floor_ms'], r['frac_of_latency_floor'], 'cpu', d['cpu_baseline']['value']);print(json.dumps(d['sw_band_opt_in']))"
