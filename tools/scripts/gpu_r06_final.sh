#!/bin/bash
# Round 6 final measurement: smoke and the whole GPU suite (SUITE=0 skips them), the profile of the default bench
# (kernel-trace stats + separate PMC passes), the default bench line with the opt-in banded leg, then the C3 and C4
# lines (EXTRA=0 skips them). First failure ends it.
TAG=${TAG:-r06final}
set -o pipefail
mkdir -p gpurun_out
if [ "${SUITE:-1}" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_all_$TAG.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gpu_all_$TAG.log | head; tail -5 gpurun_out/gpu_all_$TAG.log; exit 1; }
  tail -1 gpurun_out/gpu_all_$TAG.log
fi
bash tools/scripts/profile_r06.sh $TAG || { echo PROFILE_FAILED; exit 1; }
timeout -k 10 600 python -u bench.py --sw-band 16 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));b=d['breakdown'];r=d['roofline'];print('c5', d['value'], d['ms_per_step'], 'search', b['search_ms'], 'sw', b['sw_rerank_ms'], 'frac', r['frac'], 'floor', r['latency_floor_ms'], r['frac_of_latency_floor'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('sw_kind'), d['cpu_baseline'].get('sw_matches_oracle'), 'host', d['host_path']['ms'], 'enc', d['encoder']['ms'])"
if [ "${EXTRA:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --workload c3 --no-cpu > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || { echo C3_FAILED; tail -20 gpurun_out/bench_${TAG}_c3.err; exit 1; }
  timeout -k 10 900 python -u bench.py --workload c4 --no-cpu > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err || { echo C4_FAILED; tail -20 gpurun_out/bench_${TAG}_c4.err; exit 1; }
  python -c "import json;[print(w, json.load(open('gpurun_out/bench_${TAG}_'+w+'.json'))['value']) for w in ('c3','c4')]"
fi
