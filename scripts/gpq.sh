#!/bin/bash
# queue helper: run one gpurun call, re-submitting ONLY when gpurun reports
# exit 3 (no box / slot free; nothing ran, nothing charged). Any other exit ends it.
# usage: gpq.sh OUTFILE TIMEOUT CMD
out=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && { echo "rc=$rc" >> "$out"; exit $rc; }
  sleep 90
done
