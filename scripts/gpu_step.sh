#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call after a
# timeout / abort / segfault (exit 124, 137, 134, 139) — test failures (1) continue.
# usage: scripts/gpu_step.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc : $*" >> "$log"
case $rc in
  124|137|134|139|143) echo "FATAL rc=$rc in: $*"; exit $rc;;
esac
exit 0
