#!/bin/bash
# C3 CLI timeline: bin/pipeline with the executor trace, then under rocprofv3 kernel + copy traces
# (gpurun_out/pipe_prof/*.csv; tools/scripts/timeline.py prints the timed window)
set -o pipefail
mkdir -p gpurun_out
DRM_EXEC_VERBOSE=1 timeout -k 10 300 python -u tools/scripts/pipeline_c3.py > gpurun_out/pipeline_c3.txt 2>&1 || { tail -20 gpurun_out/pipeline_c3.txt; exit 1; }
grep -E "run |Search|device span|batch 0 enq" gpurun_out/pipeline_c3.txt
cd /tmp/drm_pipeline_c3 && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pipe_prof -o pipe --output-format csv -- $GRAFT_REPO_ROOT/bin/pipeline c3idx c3.fastq c3.fna 128 128 5 out > $GRAFT_REPO_ROOT/gpurun_out/pipe_prof.log 2>&1
