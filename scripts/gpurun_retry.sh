#!/bin/bash
# usage: gpurun_retry.sh <outfile> <timeout> <command>; re-submits only while no box/slot is free (status transient)
out=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q '"status": "transient"' /root/repo/gpurun_out/.last_call.json 2>/dev/null && [ $rc -ne 0 ]; then
    echo "[retry $i: no slot]" >> $out.retries; sleep 120; continue
  fi
  break
done
echo "RC=$rc" >> $out
