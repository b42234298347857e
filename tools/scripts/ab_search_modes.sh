set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests_3.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_3.log; exit 1; }
tail -2 gpurun_out/gpu_tests_3.log
DRM_SEARCH_LDS_KERNEL=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k search > gpurun_out/gpu_tests_3b.log 2>&1 || { echo LDS_TESTS_FAILED; tail -20 gpurun_out/gpu_tests_3b.log; exit 1; }
for cfg in "1 1" "1 0" "0 1" "0 0"; do set -- $cfg
  DRM_SEARCH_VMODE=$1 DRM_SEARCH_SPEC=$2 timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/ab_$1_$2.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ab_$1_$2.json'));print('vmode=$1 spec=$2', d['value'], d['breakdown']['search_ms'], d['breakdown']['sw_rerank_ms'], d['roofline']['frac'])"
done
