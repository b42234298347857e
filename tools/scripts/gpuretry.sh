#!/bin/bash
# Resubmit a gpurun call while the pool reports a transient refusal (no free box or slot, a box lost while being
# prepared: nothing ran on the GPU, nothing was charged). A call whose command ran is never resubmitted.
# Usage: bash tools/scripts/gpuretry.sh OUT_FILE gpurun-args...
OUT=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $OUT; then echo "rc=$rc after $i tries" >> $OUT; exit $rc; fi
  sleep 120
done
