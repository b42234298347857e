#!/bin/bash
# round-end rehearsal: the full GPU suite, smoke(), the default bench (C5) and a C3 bench (stand-in search, GRU L2)
TAG=${TAG:-r02m}
set -o pipefail
bash tools/scripts/gpu_full.sh || exit 1
timeout -k 10 600 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || { echo C3_BENCH_FAILED; tail -20 gpurun_out/bench_${TAG}_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_c3.json'));print('c3', d['value'], d['l2_rerank']['ms'], d['l2_rerank']['truth_top1'])"
