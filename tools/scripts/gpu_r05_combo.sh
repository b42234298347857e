#!/bin/bash
# Round 5: search A/B (libraries after --sw are SW-probe A/B libraries), then smoke, the whole GPU suite and the default
# bench line on the in-tree build. First failure ends it. Usage: TAG=... gpu_r05_combo.sh search_lib ... --sw sw_lib ...
TAG=${TAG:-r05}
set -o pipefail
mkdir -p gpurun_out
S=(); W=(); dst=S
for x in "$@"; do if [ "$x" = "--sw" ]; then dst=W; continue; fi; if [ $dst = S ]; then S+=("$x"); else W+=("$x"); fi; done
if [ ${#S[@]} -gt 0 ]; then
  bash tools/scripts/ab_search.sh $TAG "${S[@]}" > gpurun_out/ab_search_$TAG.txt 2>&1 || { echo AB_SEARCH_FAILED; tail -5 gpurun_out/ab_search_$TAG.txt; exit 1; }
  cat gpurun_out/ab_search_$TAG.txt
fi
if [ ${#W[@]} -gt 0 ]; then
  bash tools/scripts/ab_sw.sh "${W[@]}" > gpurun_out/ab_sw_$TAG.txt 2>&1 || { echo AB_SW_FAILED; tail -5 gpurun_out/ab_sw_$TAG.txt; exit 1; }
  cat gpurun_out/ab_sw_$TAG.txt
fi
if [ "${FULL:-1}" = "1" ]; then TAG=$TAG bash tools/scripts/gpu_r05_full.sh; fi
