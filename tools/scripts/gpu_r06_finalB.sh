#!/bin/bash
# Round 6 final call B: the C3 and C4 bench lines, (the N = 2 rehearsal runs in a call of its own: gpu_2rank_rehearsal.sh).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06final}
timeout -k 10 600 python -u bench.py --workload c3 --no-cpu > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || { echo C3_FAILED; tail -20 gpurun_out/bench_${TAG}_c3.err; exit 1; }
timeout -k 10 600 python -u bench.py --workload c4 --no-cpu > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err || { echo C4_FAILED; tail -20 gpurun_out/bench_${TAG}_c4.err; exit 1; }
python -c "import json;[print(w, json.load(open('gpurun_out/bench_${TAG}_'+w+'.json'))['value']) for w in ('c3','c4')]"
