#!/bin/bash
# retry a gpurun call while the pool has no free box (exit 3: nothing ran, nothing charged)
OUT=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "has no free box right now" $OUT; then echo "rc=$rc after $i tries" >> $OUT; exit $rc; fi
  sleep 150
done
