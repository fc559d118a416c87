#!/bin/bash
# (client side, in the build container: never uploaded, listed in .gpurunignore)
# retry a gpurun call while the pool has no free box (status transient / exit 3); nothing ran in those attempts
out=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out && ! grep -q "status=ok\|status=failed" $out; then
    sleep 100; continue
  fi
  exit $rc
done
exit 3
