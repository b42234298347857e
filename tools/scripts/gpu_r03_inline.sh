set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -m gpu -k "not c4 and not flat" > gpurun_out/r03g_tests.log 2>&1 || { tail -30 gpurun_out/r03g_tests.log; exit 1; }
tail -2 gpurun_out/r03g_tests.log
for r in 1 2; do for inl in 0 1; do DRM_SEARCH_INLINE=$inl timeout -k 10 600 python -u tools/scripts/search_c5.py 2>&1 | grep "^search" || exit 1; done; done
DRM_SEARCH_INLINE=1 timeout -k 10 600 python -u tools/scripts/search_c5.py --k 5 2>&1 | grep "^search"
DRM_SEARCH_INLINE=0 timeout -k 10 600 python -u tools/scripts/search_c5.py --k 5 2>&1 | grep "^search"
