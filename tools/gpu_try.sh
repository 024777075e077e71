#!/bin/bash
# Run one gpurun call; when the GPU service reports a transient
# infrastructure condition (no box free, box taken away before the command
# ran -- .last_call.json status "transient", nothing charged), wait and ask
# again, up to 12 times.  A command that ran and failed is never retried.
#   tools/gpu_try.sh TIMEOUT_S script.sh
set -u
t=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gpu_try] transient (try $i), waiting 150 s"
  sleep 150
done
exit 3
