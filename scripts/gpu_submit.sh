#!/bin/bash
# usage: gpu_submit.sh <tag> <timeout> <command...>; retries only while no GPU slot is free
tag=$1; to=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > gpurun_out/${tag}_call.log 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|slot(s) on this pod are busy" gpurun_out/${tag}_call.log && [ $rc -ne 0 ] && ! grep -q "status=fail\|status=ok" gpurun_out/${tag}_call.log; then
    sleep 150; continue
  fi
  break
done
echo "done rc=$rc" >> gpurun_out/${tag}_call.log
