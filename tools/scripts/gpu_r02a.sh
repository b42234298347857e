set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_r02a.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_r02a.log; exit 1; }
tail -3 gpurun_out/gpu_tests_r02a.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_r02a.json 2> gpurun_out/bench_r02a.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_r02a.err; exit 1; }
cat gpurun_out/bench_r02a.json
