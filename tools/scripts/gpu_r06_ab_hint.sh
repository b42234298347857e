#!/bin/bash
# Round 6: pop_min's hint check as one scalar select (ab_live/v1hint.so: 1 SALU fewer per hop) vs the final build, C5
# search, two rounds on one box.
set -o pipefail
mkdir -p gpurun_out/r06_ab
bash tools/scripts/ab_search.sh r06hint deepreadmapper_amd/libdrm_hip.so ab_live/v1hint.so | tee gpurun_out/r06_ab/ab_search_hint.txt
